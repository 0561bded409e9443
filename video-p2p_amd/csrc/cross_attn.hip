// K2 — hooked cross-attention over the <=128 text tokens with the P2P edit fused into the softmax
// epilogue.
//
// Reference path (one call per attn2 layer, 16 per UNet forward):
//   ptp_utils.py:206-220   q/k/v heads->batch, sim = q k^T * scale, softmax, controller, attn @ v
//   run_videop2p.py:212-224  the controller edits only the conditional half attn[h//2:]
//   run_videop2p.py:304-317  AttentionControlEdit.forward: per word w of each edited prompt
//        new[w] = alpha_t[w] * R[w] + (1 - alpha_t[w]) * P_edit[w]
//        R      = Replace: sum_j P_src[j] * M[j, w]                           (:333-334)
//                 Refine : P_src[mapper[w]] * a[w] + P_edit[w] * (1 - a[w])   (:344-347)
//                 Reweight wraps either: R * eq[w]                            (:359-363)
//   run_videop2p.py:255-268  AttentionStore keeps the post-edit conditional maps (N <= 32^2),
//        summed over steps; LocalBlend only ever reads sum_w alpha_lb[p][w] * maps of the res-16
//        layers (:131-146), so this kernel accumulates exactly that reduction (lb_acc) instead.
//
// The reference materialises probs (B*f*h, N, 77) and makes ~6-8 elementwise passes over them.
// Here one wave owns 32 query tokens x one head of one CFG half for all its prompts: the source
// prompt's probabilities are parked in LDS (fp32) while the edited prompts are computed, so the
// edit is a handful of LDS reads per word and nothing but Q in / O out touches HBM.
// The 77-token K/V (identical for all frames: attention.py:95 repeats the context per frame) are
// pre-laid-out once per layer by vp2p_cross_kv_prep into MFMA fragment order and read through L1/L2.
#include <stdlib.h>

#include <algorithm>

#include "common.hpp"
#include "vp2p.h"

namespace vp2p {

template <typename T, int D>
struct CrossCfg {
  static constexpr bool BF = sizeof(T) == 2;
  static constexpr int KD = Mfma<T>::KD;
  static constexpr int DP = round_up(D, KD);
  static constexpr int KS = DP / KD;
  static constexpr int DV = round_up(D, 32);
  static constexpr int NT = DV / 32;
  static constexpr int OCC = !BF ? 1 : (D <= 80 ? 3 : 2);   // waves/SIMD requested (no spills at 3 for these)
};

// Workspace layout for KB key blocks (KP = 32*KB padded keys), per (b, head):
//   K  : [KP][DP]  zero padded                                  (row = key)
//   V  : bf16 -> [DV][KP] with keys permuted inside each 16-key group so that one lane's PV
//                 A fragment (keys 8(j>>2) + 4h + (j&3), j = 0..7) is 16 contiguous bytes
//        f32  -> [KP][DV] row-major
template <typename T>
__host__ __device__ inline int64_t cross_ws_elems(int batch, int heads, int kp, int dp, int dv) {
  return (int64_t)batch * heads * kp * (dp + dv);
}

template <typename T, int D>
__global__ void cross_kv_prep_kernel(const T* __restrict__ k, const T* __restrict__ v, int64_t k_sb,
                                     int64_t k_sn, int64_t v_sb, int64_t v_sn, int batch, int nkv,
                                     int heads, int kp, T* __restrict__ ws) {
  using C = CrossCfg<T, D>;
  const int64_t kelems = (int64_t)batch * heads * kp * C::DP;
  const int64_t total = kelems + (int64_t)batch * heads * kp * C::DV;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    T val = (T)0.f;
    if (i < kelems) {
      const int c = (int)(i % C::DP);
      const int64_t rowi = i / C::DP;
      const int key = (int)(rowi % kp);
      const int bh = (int)(rowi / kp);
      const int b = bh / heads, head = bh % heads;
      if (key < nkv && c < D) val = k[b * k_sb + key * k_sn + head * D + c];
    } else {
      const int64_t j = i - kelems;
      int key, c, bh;
      if constexpr (C::BF) {
        const int slot = (int)(j % kp);
        const int64_t rowi = j / kp;
        c = (int)(rowi % C::DV);
        bh = (int)(rowi / C::DV);
        const int grp = slot >> 4, pos = slot & 15, hh = pos >> 3, jj = pos & 7;
        key = 16 * grp + 8 * (jj >> 2) + 4 * hh + (jj & 3);
      } else {
        c = (int)(j % C::DV);
        const int64_t rowi = j / C::DV;
        key = (int)(rowi % kp);
        bh = (int)(rowi / kp);
      }
      const int b = bh / heads, head = bh % heads;
      if (key < nkv && c < D) val = v[b * v_sb + key * v_sn + head * D + c];
    }
    ws[i] = val;
  }
}

// One wave owns one (CFG half, 32-query block, head) item at a time and walks the half's prompts in
// order, so the source prompt's probabilities (parked in the wave's LDS rows) are there when the
// edited prompts need them.  A workgroup (4 waves = 4 heads) of CFG half blockIdx.y takes items
// blockIdx.x, + gridDim.x, ..., and every wave fetches the next (item, prompt)'s Q fragments while
// the current one computes.  Waves never synchronise after the table staging; the
// LocalBlend head sum is finished by cross_lb_reduce_kernel from per-head partials, in head order.
template <typename T, int D, int KB>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(CrossCfg<T, D>::OCC, 8)))
void cross_attn_kernel(const vp2p_cross_attn_args a, int prow, int g0) {
  using M = Mfma<T>;
  using C = CrossCfg<T, D>;
  constexpr int KP = 32 * KB;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x, l = tid & 63, w = tid >> 6, r = l & 31, h = l >> 5;
  const int FQ = a.frames * a.tokens_q;
  const int qblocks = (FQ + 31) >> 5;
  const int hgroups = (a.heads + 3) >> 2;
  const int items = qblocks * hgroups;
  const bool p2p = a.prompts > 0 && a.batch == (a.cond_only ? 1 : 2) * a.prompts;
  const int RP = p2p ? a.prompts : 1;          // rows per group
  const int g = g0 + (int)blockIdx.y;          // group: CFG half (p2p) or batch row
  const bool cond = p2p && (a.cond_only || g == 1);   // cond_only: the one group is the conditional half
  const bool edit = cond && (a.edit_mode != VP2P_EDIT_NONE || a.reweight);
  const bool lb = cond && a.lb_acc != nullptr;
  const int NKV = a.tokens_kv;

  float* psrc = reinterpret_cast<float*>(smem) + (w * 32 + r) * prow;
  // The edit tables of this CFG half, staged once per workgroup (every lane of a 32-lane half reads
  // the same word, so these are broadcast LDS reads): per edited prompt and word
  // {refine alpha, equalizer, alpha_t, source word}, and LocalBlend's word weights per prompt.
  f32x4* etab = reinterpret_cast<f32x4*>(reinterpret_cast<float*>(smem) + 4 * 32 * prow);
  float* lbw = reinterpret_cast<float*>(etab + (a.prompts > 1 ? (a.prompts - 1) * NKV : 0));
  if (edit) {
    for (int i = tid; i < (RP - 1) * NKV; i += 256) {
      const int wd = i % NKV;
      f32x4 t;
      t[0] = a.edit_mode == VP2P_EDIT_REFINE ? a.refine_alpha[i] : 0.f;
      t[1] = a.reweight ? a.equalizer[wd] : 1.f;
      t[2] = a.alpha_words[i];
      t[3] = __int_as_float(a.edit_mode == VP2P_EDIT_REFINE ? a.map_idx[i] : wd);
      etab[i] = t;
    }
  }
  const int LBS = a.lb_sets == 2 ? 2 : 1;     // word-weight sets: blend words (+ substruct words)
  if (lb)
    for (int i = tid; i < LBS * RP * NKV; i += 256) lbw[i] = a.lb_word_alpha[i];
  if (edit || lb) __syncthreads();

  const float cs = a.scale * kLog2e;
  const T* ws = static_cast<const T*>(a.kv_ws);
  const int64_t kelems = (int64_t)a.batch * a.heads * KP * C::DP;

  // Q fragments of (item, prompt p); zero for padded queries / heads
  auto load_q = [&](int item, int p, typename M::frag* dst) {
    const int qb = item / hgroups, head = (item - qb * hgroups) * 4 + w;
    const int qi = qb * 32 + r;
    const bool ok = qi < FQ && head < a.heads;
    const int fr = ok ? qi / a.tokens_q : 0;
    const int pos = ok ? qi - fr * a.tokens_q : 0;
    const T* row = static_cast<const T*>(a.q) + (g * RP + p) * a.q_sb + fr * a.q_sf + pos * a.q_sn + head * D;
#pragma unroll
    for (int s = 0; s < C::KS; ++s) dst[s] = ok ? M::row_frag(row, s, h, D) : M::zero();
  };

  typename M::frag qn[C::KS];
  if (blockIdx.x < items) load_q(blockIdx.x, 0, qn);

  for (int item = blockIdx.x; item < items; item += gridDim.x) {
    const int qb = item / hgroups;
    const int head = (item - qb * hgroups) * 4 + w;
    const bool hv = head < a.heads;
    const int qi = qb * 32 + r;
    const bool qv = qi < FQ && hv;
    const int fr = qv ? qi / a.tokens_q : 0;
    const int pos = qv ? qi - fr * a.tokens_q : 0;
    const int hs = hv ? head : 0;              // padded heads compute on head 0's K/V, store nothing
  for (int p = 0; p < RP; ++p) {
    const int b = g * RP + p;
    typename M::frag qf[C::KS];
#pragma unroll
    for (int s = 0; s < C::KS; ++s) qf[s] = qn[s];
    if (p + 1 < RP) load_q(item, p + 1, qn);
    else if (item + (int)gridDim.x < items) load_q(item + gridDim.x, 0, qn);

    const T* kb_base = ws + ((int64_t)(b * a.heads + hs) * KP) * C::DP;
    f32x16 sc[KB];
#pragma unroll
    for (int kb = 0; kb < KB; ++kb) {
      sc[kb] = zero16();
      const T* krow = kb_base + (kb * 32 + r) * C::DP;
#pragma unroll
      for (int s = 0; s < C::KS; ++s) {
        typename M::frag af;
        if constexpr (C::BF) af = *reinterpret_cast<const bf16x8*>(krow + 16 * s + 8 * h);
        else af = krow[2 * s + h];
        sc[kb] = M::mma(af, qf[s], sc[kb]);
      }
    }
    // row softmax over the valid keys (the reference's global max gives the same probabilities
    // wherever it does not underflow: ptp_utils.py:217)
    float mx = kNegInf;
#pragma unroll
    for (int kb = 0; kb < KB; ++kb)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const float v = (kb * 32 + acc_row(i, h) < NKV) ? sc[kb][i] * cs : kNegInf;
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
    for (int kb = 0; kb < KB; ++kb)
#pragma unroll
      for (int i = 0; i < 16; ++i) sc[kb][i] *= inv;

    if (edit) {
      if (p == 0) {
#pragma unroll
        for (int kb = 0; kb < KB; ++kb)
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const int wd = kb * 32 + acc_row(i, h);
            if (wd < NKV) psrc[wd] = sc[kb][i];
          }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      } else {
#pragma clang fp contract(off)
        const int pe = p - 1;
#pragma unroll
        for (int kb = 0; kb < KB; ++kb)
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const int wd = kb * 32 + acc_row(i, h);
            if (wd < NKV) {
              const float pe_val = sc[kb][i];
              const f32x4 t = etab[pe * NKV + wd];
              float R;
              if (a.edit_mode == VP2P_EDIT_REPLACE) {
                const int* ptr = a.map_ptr + pe * (NKV + 1);
                float gsum = 0.f;
                for (int n = ptr[wd]; n < ptr[wd + 1]; ++n) gsum += psrc[a.map_idx[n]] * a.map_val[n];
                R = gsum;
              } else if (a.edit_mode == VP2P_EDIT_REFINE) {
                R = psrc[__float_as_int(t[3])] * t[0] + pe_val * (1.f - t[0]);
              } else {
                R = psrc[wd];
              }
              R = R * t[1];             // equalizer (1 without Reweight: exact)
              sc[kb][i] = R * t[2] + (1.f - t[2]) * pe_val;
            }
          }
      }
    }
    if (lb) {  // this head's word-weighted map of token qi -> lb_ws[set][p][head][qi]
      for (int set = 0; set < LBS; ++set) {
        const float* wts = lbw + (set * RP + p) * NKV;
        float part = 0.f;
#pragma unroll
        for (int kb = 0; kb < KB; ++kb)
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const int wd = kb * 32 + acc_row(i, h);
            if (wd < NKV) part += wts[wd] * sc[kb][i];
          }
        part += xhalf(part);
        if (h == 0 && qv) a.lb_ws[((int64_t)(set * RP + p) * a.heads + head) * FQ + qi] = part;
      }
    }
    if (a.probs_out && qv) {
      float* prow_out = a.probs_out + ((((int64_t)b * a.frames + fr) * a.heads + head) * a.tokens_q + pos) * NKV;
#pragma unroll
      for (int kb = 0; kb < KB; ++kb)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int wd = kb * 32 + acc_row(i, h);
          if (wd < NKV) prow_out[wd] = sc[kb][i];
        }
    }

    // O^T = V^T P^T over the padded keys (P is exactly 0 there)
    const T* vb_base = ws + kelems + ((int64_t)(b * a.heads + hs) * KP) * C::DV;
    f32x16 o[C::NT];
#pragma unroll
    for (int t = 0; t < C::NT; ++t) o[t] = zero16();
#pragma unroll
    for (int kb = 0; kb < KB; ++kb)
#pragma unroll
      for (int sp = 0; sp < M::PV_STEPS; ++sp) {
        const typename M::frag pf = M::p_frag(sc[kb], sp);
#pragma unroll
        for (int t = 0; t < C::NT; ++t) {
          typename M::frag vf;
          if constexpr (C::BF)
            vf = *reinterpret_cast<const bf16x8*>(vb_base + (int64_t)(32 * t + r) * KP + kb * 32 + 16 * sp + 8 * h);
          else
            vf = vb_base[(int64_t)(kb * 32 + f32_pv_key(sp, h)) * C::DV + 32 * t + r];
          o[t] = M::mma(vf, pf, o[t]);
        }
      }
    if (qv) {
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
}

// ------------------------------------------------------------------------------------------------
// K2 v3 (bf16, any head dim): the launches WITHOUT an edit, K/V of one (batch row, head) in LDS.
//
// A workgroup is one (batch row, head): its 4 waves are 4 query streams that share the row's K and
// V^T fragments, staged once from the prepared workspace into padded LDS rows (row strides of 4
// (mod 8) dwords: the 16-lane groups of a ds_read_b128 hit distinct banks).  With the fragments in
// LDS instead of registers (round-2 v2 kept them in VGPRs, d <= 64 only) and one 32-column output
// tile live at a time, a wave needs ~100 (d 40) / ~135 (d 80) VGPRs: 3-4 waves per SIMD hide the
// per-block Q -> QK^T -> softmax -> PV -> O chain and the Q fetch.  Per block only Q (prefetched one
// block ahead) comes in and O goes out.  Measured (profiles/r02_k2_v3_ab.jsonl, non-edit launches,
// B4 f8): res-64 d 40 54.9 (v2) -> 53.9 us, res-32 d 80 62.0 (v1) -> 39.5, res-16 d 160 37.4 -> 26.5.
// ------------------------------------------------------------------------------------------------
template <int D, int KB>
struct CrossV3Cfg {
  using C = CrossCfg<bf16, D>;
  static constexpr int KP = 32 * KB;
  static constexpr int KROW = C::DP + 8;          // K rows (keys) in LDS
  static constexpr int VROW = KP + 8;             // V^T rows (head columns) in LDS
  static constexpr int LDS = (KP * KROW + C::DV * VROW) * 2;
};

// Staging of the prepared K [KP][DP] / V^T [DV][KP] fragments into padded LDS rows.  A segment is N
// contiguous 16-byte vectors of the workspace whose rows of RV vectors land RS vectors apart in LDS;
// a thread's vectors are i = tid + j * NT.  All of a thread's loads of the segments it is given go
// out before its stores (a load-then-store loop waits out one L2 latency per vector), and the
// addressing is one multiply-high per vector (the per-vector (prompt, K | V, row) decode it replaced
// was ~60 % of v3e's VALU instructions at d = 160).
template <int NT, int N, int RV, int RS>
struct StageSeg {
  static constexpr int PER = (N + NT - 1) / NT;
  const u32x4* src;
  u32x4* dst;
  u32x4 buf[PER];
  __device__ __forceinline__ void load(int tid) {
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int i = tid + j * NT;
      if (N % NT == 0 || i < N) buf[j] = src[i];
    }
  }
  __device__ __forceinline__ void store(int tid) {
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int i = tid + j * NT;
      if (N % NT == 0 || i < N) dst[i + (i / RV) * (RS - RV)] = buf[j];
    }
  }
};

// T77: the SD text context (77 tokens, KB = 3): in the last 32-key block only keys 64..76 are real,
// so accumulator registers 8..15 (keys 80..95 for both lane halves) are never computed through exp
// and the block's second PV k-step (keys 80..95) is skipped.
// MODE 0: Q fragments loaded straight from HBM one block ahead;
// 2 ("staged", needs tokens_q % 32 == 0): a wave moves its block's Q rows and O rows as whole
// 2d-byte row segments (5 / 10 / 20 lanes per row for d = 40 / 80 / 160) through a private LDS
// tile, instead of fragment-shaped loads / stores that touch 32 rows x 16-32 B per instruction.
template <int D, int KB, bool T77 = false, int MODE = 0>
__global__ __launch_bounds__(256, D <= 64 ? 3 : 2) void cross_attn_kernel_v3(const vp2p_cross_attn_args a, int iters, int b0,
                                                                               int nx, int rows) {
  static_assert(MODE == 0 || MODE == 2, "Q path");
  constexpr bool STG = MODE == 2;
  using T = bf16;
  using M = Mfma<T>;
  using C = CrossCfg<T, D>;
  using V3 = CrossV3Cfg<D, KB>;
  constexpr int KP = V3::KP;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  T* Ks = reinterpret_cast<T*>(smem);
  T* Vs = Ks + KP * V3::KROW;
  float* lbw = reinterpret_cast<float*>(smem + V3::LDS);   // [sets][NKV] of this row's prompt
  const int tid = threadIdx.x, l = tid & 63, w = tid >> 6, r = l & 31, h = l >> 5;
  const int FQ = a.frames * a.tokens_q;
  const bool p2p = a.prompts > 0 && a.batch == (a.cond_only ? 1 : 2) * a.prompts;
  // 1-D grid, XCD-grouped (xcd_remap) with the head fastest: the a.heads workgroups of one query range
  // run together on ONE XCD, so the 128-B lines their head slices share (d = 40: 80-B slices of
  // 640-B rows) are fetched into one L2 once and written back whole, not once per XCD / half-written
  // (r02 PMC: 1.27x the algorithmic bytes with the (x, row, head) 3-D grid).  nx = 0: the 3-D grid.
  int bx, by, bz;
  if (nx > 0) {
    const int lid = xcd_remap((int)blockIdx.x, nx * rows * a.heads);
    bz = lid % a.heads;
    const int rest = lid / a.heads;
    bx = rest % nx;
    by = rest / nx;
  } else {
    bx = blockIdx.x, by = blockIdx.y, bz = blockIdx.z;
  }
  const int b = b0 + by;                       // batch row
  const int head = bz;
  const int g = p2p ? b / a.prompts : 0;        // CFG half
  const int pw = p2p ? b - g * a.prompts : 0;   // prompt within the half
  const bool cond = p2p && (a.cond_only || g == 1);
  const bool lb = cond && a.lb_acc != nullptr;
  const int NKV = a.tokens_kv;
  const int LBS = a.lb_sets == 2 ? 2 : 1;

  // stage this (row, head)'s K [KP][DP] and V^T [DV][KP] fragments (16-byte vectors)
  const T* ws = static_cast<const T*>(a.kv_ws);
  const int64_t kelems = (int64_t)a.batch * a.heads * KP * C::DP;
  const T* kb_base = ws + ((int64_t)(b * a.heads + head) * KP) * C::DP;
  const T* vb_base = ws + kelems + ((int64_t)(b * a.heads + head) * KP) * C::DV;
  constexpr int KV8 = KP * C::DP / 8, VV8 = C::DV * KP / 8;
  {
    StageSeg<256, KV8, C::DP / 8, V3::KROW / 8> ks{reinterpret_cast<const u32x4*>(kb_base), reinterpret_cast<u32x4*>(Ks)};
    StageSeg<256, VV8, KP / 8, V3::VROW / 8> vs{reinterpret_cast<const u32x4*>(vb_base), reinterpret_cast<u32x4*>(Vs)};
    ks.load(tid);
    vs.load(tid);
    ks.store(tid);
    vs.store(tid);
  }
  if (lb)
    for (int i = tid; i < LBS * NKV; i += 256) {
      const int set = i / NKV, wd = i - set * NKV;
      lbw[i] = a.lb_word_alpha[(set * a.prompts + pw) * NKV + wd];
    }
  __syncthreads();

  const float cs = a.scale * kLog2e;
  const bool norm_p = lb || a.probs_out;
  // stream w's query blocks: qb0, qb0 + 4, ...; (frame, token) of the lane's query tracked
  // incrementally (no integer division in the loop)
  const int qb0 = bx * 4 * iters + w;
  constexpr int NS = 4;
  const int step = 32 * NS;
  const T* qbase = static_cast<const T*>(a.q) + b * a.q_sb + head * D;
  T* obase = static_cast<T*>(a.o) + b * a.o_sb + head * D;
  int qi = qb0 * 32 + r;
  int fr = qi / a.tokens_q, pos = qi - (qi / a.tokens_q) * a.tokens_q;
  auto advance = [&](int& f_, int& p_) {
    p_ += step;
    while (p_ >= a.tokens_q) { p_ -= a.tokens_q; ++f_; }
  };
  auto load_q = [&](int qi_, int f_, int p_, bf16x8* dst) {
    const bool ok = qi_ < FQ;
    const T* row = qbase + (ok ? f_ * a.q_sf + p_ * a.q_sn : 0);
#pragma unroll
    for (int s = 0; s < C::KS; ++s) dst[s] = ok ? M::row_frag(row, s, h, D) : M::zero();
  };
  // staged mode: this wave's LDS tile (32 rows x QROW, columns D..DP-1 zero) and its row-segment chunks
  constexpr int QROW = C::DP + 8, CPR = D / 8, NCHK = (32 * CPR + 63) / 64;
  T* Qs = reinterpret_cast<T*>(smem + V3::LDS + ((LBS * NKV * 4 + 15) & ~15)) + w * 32 * QROW;
  u32x4 qraw[STG ? NCHK : 1];
  auto load_raw = [&](int qi_, int f_, int p_) {        // the block of lane row r = qi_ (frame f_, token p_)
    const int q0 = qi_ - r, n0 = p_ - r;                // tokens_q % 32 == 0: the block sits in frame f_
#pragma unroll
    for (int i = 0; i < NCHK; ++i) {
      const int c = i * 64 + l, row = c / CPR, ch = c - row * CPR;
      qraw[i] = (c < 32 * CPR && q0 + row < FQ)
                    ? *reinterpret_cast<const u32x4*>(qbase + f_ * a.q_sf + (n0 + row) * a.q_sn + ch * 8)
                    : u32x4{0, 0, 0, 0};
    }
  };
  if constexpr (STG) {
    if constexpr (C::DP > D)
      for (int i = l; i < 32 * (C::DP - D); i += 64) {
        const int row = i / (C::DP - D);
        Qs[row * QROW + D + (i - row * (C::DP - D))] = (T)0.f;
      }
  }
  bf16x8 qn[C::KS];
  if constexpr (STG) load_raw(qi, fr, pos);
  else load_q(qi, fr, pos, qn);
  int fr_n = fr, pos_n = pos;          // (frame, token) of block qi

  for (int it = 0; it < iters; ++it) {
    bf16x8 qf[C::KS];
    if constexpr (STG) {
      // this block's row segments -> LDS (the wave's own tile: LDS ops of one wave stay in order)
#pragma unroll
      for (int i = 0; i < NCHK; ++i) {
        const int c = i * 64 + l, row = c / CPR, ch = c - row * CPR;
        if (c < 32 * CPR) *reinterpret_cast<u32x4*>(Qs + row * QROW + ch * 8) = qraw[i];
      }
    } else {
#pragma unroll
      for (int s = 0; s < C::KS; ++s) qf[s] = qn[s];
    }
    const int qcur = qi;
    const int fcur = fr_n, pcur = pos_n;
    if constexpr (STG) {
      if (it + 1 < iters) {
        advance(fr_n, pos_n);
        qi += step;
        load_raw(qi, fr_n, pos_n);
      }
#pragma unroll
      for (int s = 0; s < C::KS; ++s) qf[s] = *reinterpret_cast<const bf16x8*>(Qs + r * QROW + 16 * s + 8 * h);
    } else if (it + 1 < iters) {
      advance(fr_n, pos_n);
      qi += step;
      load_q(qi, fr_n, pos_n, qn);
    }
    const bool qv = qcur < FQ;

    f32x16 sc[KB];
#pragma unroll
    for (int kb = 0; kb < KB; ++kb) {
      sc[kb] = zero16();
#pragma unroll
      for (int s = 0; s < C::KS; ++s)
        sc[kb] = M::mma(*reinterpret_cast<const bf16x8*>(Ks + (kb * 32 + r) * V3::KROW + 16 * s + 8 * h), qf[s], sc[kb]);
      __builtin_amdgcn_sched_barrier(0);      // no hoisting of every block's K fragments at once
    }
    // row softmax: only the last key block is ragged; max on raw scores, exp2(s*cs - max*cs) fused
    float mx = kNegInf;
#pragma unroll
    for (int kb = 0; kb < KB; ++kb)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        if (T77 && kb == KB - 1 && i >= 8) continue;
        if (kb == KB - 1 && kb * 32 + acc_row(i, h) >= NKV) sc[kb][i] = kNegInf;
        mx = fmaxf(mx, sc[kb][i]);
      }
    mx = fmaxf(mx, xhalf(mx)) * cs;
    float sum = 0.f;
#pragma unroll
    for (int kb = 0; kb < KB; ++kb)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        if (T77 && kb == KB - 1 && i >= 8) {
          sc[kb][i] = 0.f;
          continue;
        }
        const float e = fast_exp2(__builtin_fmaf(sc[kb][i], cs, -mx));
        sc[kb][i] = e;
        sum += e;
      }
    sum += xhalf(sum);
    const float inv = 1.f / sum;
    if (norm_p) {
#pragma unroll
      for (int kb = 0; kb < KB; ++kb)
#pragma unroll
        for (int i = 0; i < 16; ++i) sc[kb][i] *= inv;
      if (lb) {  // this head's word-weighted map of token qi -> lb_ws[set][p][head][qi]
        for (int set = 0; set < LBS; ++set) {
          const float* wts = lbw + set * NKV;
          float part = 0.f;
#pragma unroll
          for (int kb = 0; kb < KB; ++kb)
#pragma unroll
            for (int i = 0; i < 16; ++i) {
              const int wd = kb * 32 + acc_row(i, h);
              if (wd < NKV) part += wts[wd] * sc[kb][i];
            }
          part += xhalf(part);
          if (h == 0 && qv) a.lb_ws[((int64_t)(set * a.prompts + pw) * a.heads + head) * FQ + qcur] = part;
        }
      }
      if (a.probs_out && qv) {
        float* prow_out = a.probs_out + ((((int64_t)b * a.frames + fcur) * a.heads + head) * a.tokens_q + pcur) * NKV;
#pragma unroll
        for (int kb = 0; kb < KB; ++kb)
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const int wd = kb * 32 + acc_row(i, h);
            if (wd < NKV) prow_out[wd] = sc[kb][i];
          }
      }
    }
    const float oscale = norm_p ? 1.f : inv;
    // P as bf16 B fragments (the fp32 scores die here), then one 32-column output tile at a time:
    // only 16 accumulators live, which keeps d = 80 / 160 within the register budget
    bf16x8 pf[KB][2];
#pragma unroll
    for (int kb = 0; kb < KB; ++kb) {
      pf[kb][0] = M::p_frag(sc[kb], 0);
      pf[kb][1] = M::p_frag(sc[kb], 1);
    }
    T* orow = obase + fcur * a.o_sf + pcur * a.o_sn;
#pragma unroll
    for (int t = 0; t < C::NT; ++t) {
      f32x16 o = zero16();
#pragma unroll
      for (int kb = 0; kb < KB; ++kb)
#pragma unroll
        for (int sp = 0; sp < 2; ++sp) {
          if (T77 && kb == KB - 1 && sp == 1) continue;     // keys 80..95: no context tokens
          o = M::mma(*reinterpret_cast<const bf16x8*>(Vs + (32 * t + r) * V3::VROW + kb * 32 + 16 * sp + 8 * h), pf[kb][sp], o);
        }
      __builtin_amdgcn_sched_barrier(0);
      if (STG || qv) {
#pragma unroll
        for (int gq = 0; gq < 4; ++gq) {
          const int dc = 32 * t + 8 * gq + 4 * h;
          if (dc < D) {
            bf16x4 v;
#pragma unroll
            for (int j = 0; j < 4; ++j) v[j] = (bf16)(o[4 * gq + j] * oscale);
            if constexpr (STG) *reinterpret_cast<bf16x4*>(Qs + r * QROW + dc) = v;
            else *reinterpret_cast<bf16x4*>(orow + dc) = v;
          }
        }
      }
    }
    if constexpr (STG) {     // the block's O rows out of the LDS tile as whole row segments
      const int q0 = qcur - r, n0 = pcur - r;
      T* ob = obase + fcur * a.o_sf;
#pragma unroll
      for (int i = 0; i < NCHK; ++i) {
        const int c = i * 64 + l, row = c / CPR, ch = c - row * CPR;
        if (c < 32 * CPR && q0 + row < FQ)
          *reinterpret_cast<u32x4*>(ob + (n0 + row) * a.o_sn + ch * 8) =
              *reinterpret_cast<const u32x4*>(Qs + row * QROW + ch * 8);
      }
    }
  }
}


// ------------------------------------------------------------------------------------------------
// K2 v3e (bf16, prompts = 2): the EDITED conditional half of an edit launch (run_videop2p.py:304-317:
// the reference edits attn[h//2:] only), v3-style.  A workgroup is one head of the conditional half:
// both prompts' K and V^T fragments sit in LDS (staged once), and its 8 waves are 8 query streams.
// Per query block a wave computes the source prompt (its probabilities parked in the wave's own LDS
// rows, fp32), then the edited prompt, whose softmax epilogue applies Replace / Refine, Reweight and
// the word-alpha blend exactly as cross_attn_kernel (v1) does; Q is prefetched one (block, prompt)
// ahead.  Replaces v1 on these rows (v1: K/V re-read from L2 per item, one item per workgroup).
// d = 160 (PAIR below): 4 waves, two per query stream, one per prompt.  Round 5, res-16 edit launch
// (v3 + v3e + LocalBlend reduce, tools/k2_bench.py, profiles/r05_k2_stage_ab.jsonl): 63.1 -> 38.5 us
// (v3e 52.9 -> 18.0 us: staging addressing 21 us, the prompt pairs 3 us), bit-equal.
// ------------------------------------------------------------------------------------------------
template <int D> constexpr int v3e_threads() { return D <= 80 ? 512 : 256; }
template <int D, int KB>
struct CrossV3eCfg {
  using V3 = CrossV3Cfg<D, KB>;
  // PAIR (d 160): the two prompts of a query block run on two waves at once -- the source wave parks
  // its probabilities, a workgroup barrier, the edited wave reads them -- instead of one after the
  // other on one wave.  d 160's two prompts' K / V^T take 132 KB of LDS, so a CU holds one workgroup
  // and the edit launch (res-16 / res-8: 64 / 16 query blocks per head) is a few waves per CU, each a
  // long dependent chain: splitting the prompts across waves halves the chain.  d <= 80 launches have
  // query blocks enough to fill the CU either way and keep one wave per stream (no barrier).
  static constexpr bool PAIR = D > 80;
  static constexpr int NW = D <= 80 ? 8 : 4;                      // waves
  static constexpr int NS = PAIR ? NW / 2 : NW;                   // query streams (parked-row slots)
  static constexpr int NT = 64 * NW;
  static_assert(NT == v3e_threads<D>(), "launch bound");
  static constexpr int KV = 2 * V3::LDS;                         // both prompts' K, V^T
};

template <int D, int KB, bool T77 = false>
__global__ __launch_bounds__(v3e_threads<D>(), 1) void cross_attn_kernel_v3e(const vp2p_cross_attn_args a, int iters, int nx, int prow) {
  using T = bf16;
  using M = Mfma<T>;
  using C = CrossCfg<T, D>;
  using V3 = CrossV3Cfg<D, KB>;
  using E = CrossV3eCfg<D, KB>;
  constexpr int KP = V3::KP;
  constexpr int NS = E::NS;
  constexpr bool PAIR = E::PAIR;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, l = tid & 63, w = tid >> 6, r = l & 31, h = l >> 5;
  const int sw = PAIR ? w >> 1 : w;                              // this wave's query stream
  const int role = PAIR ? w & 1 : 0;                             // PAIR: the prompt this wave computes
  const int NKV = a.tokens_kv;
  const int FQ = a.frames * a.tokens_q;
  const int LBS = a.lb_sets == 2 ? 2 : 1;
  const bool lb = a.lb_acc != nullptr;
  // 1-D XCD-grouped grid, head fastest (see cross_attn_kernel_v3)
  const int lid = xcd_remap((int)blockIdx.x, nx * a.heads);
  const int head = lid % a.heads, bx = lid / a.heads;
  const int brow0 = a.cond_only ? 0 : a.prompts;                // batch row of the source prompt

  T* Ks0 = reinterpret_cast<T*>(smem);
  float* psrc = reinterpret_cast<float*>(smem + E::KV) + (sw * 32 + r) * prow;
  f32x4* etab = reinterpret_cast<f32x4*>(reinterpret_cast<float*>(smem + E::KV) + NS * 32 * prow);
  float* lbw = reinterpret_cast<float*>(etab + NKV);             // [set][prompt][word]

  // stage both prompts' K [KP][DP] and V^T [DV][KP] (padded rows), the edit table and the LB weights
  const T* ws = static_cast<const T*>(a.kv_ws);
  const int64_t kelems = (int64_t)a.batch * a.heads * KP * C::DP;
  constexpr int KV8 = KP * C::DP / 8, VV8 = C::DV * KP / 8;
  // the edit of run_videop2p.py:304-317 folded per word into new = G * A + P_edit * B: G the source
  // term (Refine: P_src[mapper[w]]; Replace: sum_j P_src[j] M[j, w]; otherwise P_src[w]), A = a eq al,
  // B = (1 - a) eq al + (1 - al) (Refine; a = 0 and the (1 - a) term dropped otherwise), al = alpha_t[w],
  // eq the Reweight equalizer (1 without): one gather and one FMA per score instead of the chain
  for (int i = tid; i < NKV; i += E::NT) {
    const bool refine = a.edit_mode == VP2P_EDIT_REFINE;
    const float ra = refine ? a.refine_alpha[i] : 0.f;
    const float eq = a.reweight ? a.equalizer[i] : 1.f;
    const float al = a.alpha_words[i];
    f32x4 t;
    t[0] = (refine ? ra : 1.f) * eq * al;
    t[1] = (refine ? (1.f - ra) * eq * al : 0.f) + (1.f - al);
    t[2] = 0.f;
    t[3] = __int_as_float(refine ? a.map_idx[i] : i);
    etab[i] = t;
  }
  if (lb)
    for (int i = tid; i < LBS * 2 * NKV; i += E::NT) lbw[i] = a.lb_word_alpha[i];

  const float cs = a.scale * kLog2e;
  const int qb0 = bx * NS * iters + sw;
  constexpr int step = 32 * NS;
  int qi = qb0 * 32 + r;
  int fr_n = qi / a.tokens_q, pos_n = qi - fr_n * a.tokens_q;
  auto advance = [&](int& f_, int& p_) {
    p_ += step;
    while (p_ >= a.tokens_q) { p_ -= a.tokens_q; ++f_; }
  };
  auto load_q = [&](int qi_, int f_, int p_, int prompt, bf16x8* dst) {
    const bool ok = qi_ < FQ;
    const T* row = static_cast<const T*>(a.q) + (brow0 + prompt) * a.q_sb + head * D +
                   (ok ? f_ * a.q_sf + p_ * a.q_sn : 0);
#pragma unroll
    for (int s = 0; s < C::KS; ++s) dst[s] = ok ? M::row_frag(row, s, h, D) : M::zero();
  };
  bf16x8 qn[C::KS];
  load_q(qi, fr_n, pos_n, role, qn);     // the first Q block in flight during the staging
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const int64_t bh = (int64_t)(brow0 + p) * a.heads + head;
    T* Ks = Ks0 + p * (V3::LDS / 2);
    StageSeg<E::NT, KV8, C::DP / 8, V3::KROW / 8> ks{reinterpret_cast<const u32x4*>(ws + bh * KP * C::DP),
                                                       reinterpret_cast<u32x4*>(Ks)};
    StageSeg<E::NT, VV8, KP / 8, V3::VROW / 8> vs{reinterpret_cast<const u32x4*>(ws + kelems + bh * KP * C::DV),
                                                    reinterpret_cast<u32x4*>(Ks + KP * V3::KROW)};
    ks.load(tid);
    vs.load(tid);
    ks.store(tid);
    vs.store(tid);
  }
  __syncthreads();

  for (int it = 0; it < iters; ++it) {
    const int qcur = qi, fcur = fr_n, pcur = pos_n;
    const bool qv = qcur < FQ;
    for (int p = role; p < (PAIR ? role + 1 : 2); ++p) {
      bf16x8 qf[C::KS];
#pragma unroll
      for (int s = 0; s < C::KS; ++s) qf[s] = qn[s];
      if (PAIR) {
        if (it + 1 < iters) {
          advance(fr_n, pos_n);
          qi += step;
          load_q(qi, fr_n, pos_n, p, qn);
        }
      } else if (p == 0) {
        load_q(qcur, fcur, pcur, 1, qn);
      } else if (it + 1 < iters) {
        advance(fr_n, pos_n);
        qi += step;
        load_q(qi, fr_n, pos_n, 0, qn);
      }
      const T* Ks = Ks0 + p * (V3::LDS / 2);
      const T* Vs = Ks + KP * V3::KROW;
      f32x16 sc[KB];
#pragma unroll
      for (int kb = 0; kb < KB; ++kb) {
        sc[kb] = zero16();
#pragma unroll
        for (int s2 = 0; s2 < C::KS; ++s2)
          sc[kb] = M::mma(*reinterpret_cast<const bf16x8*>(Ks + (kb * 32 + r) * V3::KROW + 16 * s2 + 8 * h), qf[s2], sc[kb]);
        __builtin_amdgcn_sched_barrier(0);
      }
      // normalised row softmax (the edit reads probabilities: run_videop2p.py:304-317)
      float mx = kNegInf;
#pragma unroll
      for (int kb = 0; kb < KB; ++kb)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          if (T77 && kb == KB - 1 && i >= 8) continue;
          if (kb == KB - 1 && kb * 32 + acc_row(i, h) >= NKV) sc[kb][i] = kNegInf;
          mx = fmaxf(mx, sc[kb][i]);
        }
      mx = fmaxf(mx, xhalf(mx)) * cs;
      float sum = 0.f;
#pragma unroll
      for (int kb = 0; kb < KB; ++kb)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          if (T77 && kb == KB - 1 && i >= 8) {
            sc[kb][i] = 0.f;
            continue;
          }
          const float e = fast_exp2(__builtin_fmaf(sc[kb][i], cs, -mx));
          sc[kb][i] = e;
          sum += e;
        }
      sum += xhalf(sum);
      const float inv = 1.f / sum;
#pragma unroll
      for (int kb = 0; kb < KB; ++kb)
#pragma unroll
        for (int i = 0; i < 16; ++i) sc[kb][i] *= inv;

      if (p == 0) {
#pragma unroll
        for (int kb = 0; kb < KB; ++kb)
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const int wd = kb * 32 + acc_row(i, h);
            if (wd < NKV) psrc[wd] = sc[kb][i];
          }
        if (!PAIR) {
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
      }
      if (PAIR) __syncthreads();          // the source wave's rows parked -> the edited wave reads them
      if (p == 1) {
#pragma unroll
        for (int kb = 0; kb < KB; ++kb)
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const int wd = kb * 32 + acc_row(i, h);
            if (wd < NKV) {
              const f32x4 t = etab[wd];
              float G;
              if (a.edit_mode == VP2P_EDIT_REPLACE) {
                G = 0.f;
                for (int n = a.map_ptr[wd]; n < a.map_ptr[wd + 1]; ++n) G += psrc[a.map_idx[n]] * a.map_val[n];
              } else {
                G = psrc[__float_as_int(t[3])];
              }
              sc[kb][i] = __builtin_fmaf(G, t[0], sc[kb][i] * t[1]);
            }
          }
      }
      if (lb) {
        for (int set = 0; set < LBS; ++set) {
          const float* wts = lbw + (set * 2 + p) * NKV;
          float part = 0.f;
#pragma unroll
          for (int kb = 0; kb < KB; ++kb)
#pragma unroll
            for (int i = 0; i < 16; ++i) {
              const int wd = kb * 32 + acc_row(i, h);
              if (wd < NKV) part += wts[wd] * sc[kb][i];
            }
          part += xhalf(part);
          if (h == 0 && qv) a.lb_ws[((int64_t)(set * 2 + p) * a.heads + head) * FQ + qcur] = part;
        }
      }
      if (a.probs_out && qv) {
        float* prow_out = a.probs_out + ((((int64_t)(brow0 + p) * a.frames + fcur) * a.heads + head) * a.tokens_q + pcur) * NKV;
#pragma unroll
        for (int kb = 0; kb < KB; ++kb)
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const int wd = kb * 32 + acc_row(i, h);
            if (wd < NKV) prow_out[wd] = sc[kb][i];
          }
      }
      bf16x8 pf[KB][2];
#pragma unroll
      for (int kb = 0; kb < KB; ++kb) {
        pf[kb][0] = M::p_frag(sc[kb], 0);
        pf[kb][1] = M::p_frag(sc[kb], 1);
      }
      T* orow = static_cast<T*>(a.o) + (brow0 + p) * a.o_sb + head * D + fcur * a.o_sf + pcur * a.o_sn;
#pragma unroll
      for (int t = 0; t < C::NT; ++t) {
        f32x16 o = zero16();
#pragma unroll
        for (int kb = 0; kb < KB; ++kb)
#pragma unroll
          for (int sp = 0; sp < 2; ++sp) {
            if (T77 && kb == KB - 1 && sp == 1) continue;
            o = M::mma(*reinterpret_cast<const bf16x8*>(Vs + (32 * t + r) * V3::VROW + kb * 32 + 16 * sp + 8 * h), pf[kb][sp], o);
          }
        __builtin_amdgcn_sched_barrier(0);
        if (qv) {
#pragma unroll
          for (int gq = 0; gq < 4; ++gq) {
            const int dc = 32 * t + 8 * gq + 4 * h;
            if (dc < D) {
              bf16x4 v;
#pragma unroll
              for (int j = 0; j < 4; ++j) v[j] = (bf16)o[4 * gq + j];
              *reinterpret_cast<bf16x4*>(orow + dc) = v;
            }
          }
        }
      }
    }
    if (PAIR && it + 1 < iters) __syncthreads();   // the parked rows are read before they are rewritten
  }
}

// lb_acc[p][qi] += sum over heads (in head order) of lb_ws[p][head][qi]: deterministic, one
// read-modify-write per (prompt, token).
__global__ void cross_lb_reduce_kernel(float* __restrict__ lb_acc, const float* __restrict__ lb_ws,
                                       int prompts, int heads, int fq) {
  const int64_t n = (int64_t)prompts * fq;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int p = (int)(i / fq);
    const int64_t qi = i - (int64_t)p * fq;
    const float* src = lb_ws + (int64_t)p * heads * fq + qi;
    float tot = 0.f;
    for (int hd = 0; hd < heads; ++hd) tot += src[(int64_t)hd * fq];
    lb_acc[i] += tot;
  }
}

template <typename T, int D>
static int cross_dims(int& dp, int& dv) {
  dp = CrossCfg<T, D>::DP;
  dv = CrossCfg<T, D>::DV;
  return 0;
}

static int cross_pad_dims(int head_dim, int dtype, int& dp, int& dv) {
#define VP2P_DIMS(DIM) \
  case DIM: return dtype == VP2P_BF16 ? cross_dims<bf16, DIM>(dp, dv) : cross_dims<float, DIM>(dp, dv);
  switch (head_dim) {
    VP2P_DIMS(32) VP2P_DIMS(40) VP2P_DIMS(64) VP2P_DIMS(80) VP2P_DIMS(128) VP2P_DIMS(160)
    default: return VP2P_E_HEAD_DIM;
  }
#undef VP2P_DIMS
}

// v3's Q/O path (cross_attn_kernel_v3 MODE): staged rows (2) for d <= 80 -- res-64 non-edit launch
// 53.8 -> 48.5 us, res-32 edit launch 56.5 -> 53.4 us, bit-equal (profiles/r03_k2_v3_staged_ab.jsonl)
// -- and fragment loads (0) for d = 160, where the 20-lane rows cost occupancy (31.0 -> 36.4 us).
// The grid targets 4 workgroups per CU over (row, head), 1-D and XCD-grouped (measured no faster at
// 6, 8, 12 per CU, nor with two Q blocks ahead: profiles/r03_k2_v3_pf_wgcu_ab.jsonl).
constexpr int kCrossV3WgPerCu = 4;

template <typename T, int D, int KB>
static int launch_cross(const vp2p_cross_attn_args* a, hipStream_t s) {
  const int FQ = a->frames * a->tokens_q;
  // v3 over batch rows [b0, b0 + rows): every row of a non-edit launch, or the unconditional half of
  // an edit launch (the reference edits only attn[h//2:], run_videop2p.py:217-218)
  auto launch_v3 = [&](int b0, int rows) -> int {
    using V3 = CrossV3Cfg<D, KB>;
    const int64_t qblocks = (FQ + 31) / 32;
    const int64_t per_wg = (qblocks + 3) / 4;                   // iterations of one stream, all blocks
    const int64_t gh = (int64_t)rows * a->heads;
    // ~kCrossV3WgPerCu workgroups per CU over the (row, head) grid; each stream then loops `iters` blocks
    const int64_t target = 256 * kCrossV3WgPerCu;
    int64_t nx = std::max<int64_t>(1, std::min<int64_t>(per_wg, (target + gh - 1) / gh));
    const int iters = (int)((per_wg + nx - 1) / nx);
    nx = (per_wg + iters - 1) / iters;
    if (rows > 65535 || a->heads > 65535 || nx > 0x7fffffff) return VP2P_E_SHAPE;
    const int sets = a->lb_sets == 2 ? 2 : 1;
    const bool t77 = KB == 3 && a->tokens_kv == 77;
    // staged rows need whole blocks per frame
    const int mode = (D <= 80 && a->tokens_q % 32 == 0) ? 2 : 0;
    size_t lds = (size_t)V3::LDS + (size_t)sets * a->tokens_kv * sizeof(float);
    if (mode == 2) lds = ((lds + 15) & ~(size_t)15) + (size_t)4 * 32 * (CrossCfg<bf16, D>::DP + 8) * 2;
    const void* fn = nullptr;
    switch (mode + (t77 ? 1 : 0)) {
      case 0: fn = reinterpret_cast<const void*>(&cross_attn_kernel_v3<D, KB, false, 0>); break;
      case 1: fn = reinterpret_cast<const void*>(&cross_attn_kernel_v3<D, KB, true, 0>); break;
      case 2: fn = reinterpret_cast<const void*>(&cross_attn_kernel_v3<D, KB, false, 2>); break;
      default: fn = reinterpret_cast<const void*>(&cross_attn_kernel_v3<D, KB, true, 2>); break;
    }
    if (hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) != hipSuccess ||
        lds > 160 * 1024)
      return VP2P_E_LAUNCH;
    const bool g1 = nx * rows * a->heads <= 0x7fffffff;
    const dim3 grid = g1 ? dim3((unsigned)(nx * rows * a->heads)) : dim3((unsigned)nx, (unsigned)rows, (unsigned)a->heads);
    const int nx1 = g1 ? (int)nx : 0;
    switch (mode + (t77 ? 1 : 0)) {
      case 0: hipLaunchKernelGGL((cross_attn_kernel_v3<D, KB, false, 0>), grid, dim3(256), lds, s, *a, iters, b0, nx1, rows); break;
      case 1: hipLaunchKernelGGL((cross_attn_kernel_v3<D, KB, true, 0>), grid, dim3(256), lds, s, *a, iters, b0, nx1, rows); break;
      case 2: hipLaunchKernelGGL((cross_attn_kernel_v3<D, KB, false, 2>), grid, dim3(256), lds, s, *a, iters, b0, nx1, rows); break;
      default: hipLaunchKernelGGL((cross_attn_kernel_v3<D, KB, true, 2>), grid, dim3(256), lds, s, *a, iters, b0, nx1, rows); break;
    }
    return hipGetLastError() == hipSuccess ? VP2P_OK : VP2P_E_LAUNCH;
  };
  // v3e over the edited conditional half (prompts = 2, bf16); returns VP2P_E_SHAPE to fall back to v1
  auto launch_v3e = [&]() -> int {
    using V3 = CrossV3Cfg<D, KB>;
    using E = CrossV3eCfg<D, KB>;
    const int prow = a->tokens_kv | 1;
    const int sets = a->lb_sets == 2 ? 2 : 1;
    const size_t lds = (size_t)E::KV + (size_t)E::NS * 32 * prow * 4 + (size_t)a->tokens_kv * 16 +
                       (size_t)sets * 2 * a->tokens_kv * 4;
    if (lds > 160 * 1024) return VP2P_E_SHAPE;
    const int64_t qblocks = (FQ + 31) / 32;
    const int64_t per_wg = (qblocks + E::NS - 1) / E::NS;
    // ~1 workgroup per CU over the heads; each of its NS streams then loops `iters` blocks
    int64_t nx = std::max<int64_t>(1, std::min<int64_t>(per_wg, (256 + a->heads - 1) / a->heads));
    const int iters = (int)((per_wg + nx - 1) / nx);
    nx = (per_wg + iters - 1) / iters;
    if (nx * a->heads > 0x7fffffff) return VP2P_E_SHAPE;
    static const bool attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&cross_attn_kernel_v3e<D, KB>),
                                                 hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) == hipSuccess;
    static const bool attr77 = hipFuncSetAttribute(reinterpret_cast<const void*>(&cross_attn_kernel_v3e<D, KB, true>),
                                                   hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) == hipSuccess;
    if (!attr || !attr77) return VP2P_E_LAUNCH;
    const dim3 grid((unsigned)(nx * a->heads));
    if (KB == 3 && a->tokens_kv == 77)
      hipLaunchKernelGGL((cross_attn_kernel_v3e<D, KB, true>), grid, dim3(E::NT), lds, s, *a, iters, (int)nx, prow);
    else
      hipLaunchKernelGGL((cross_attn_kernel_v3e<D, KB>), grid, dim3(E::NT), lds, s, *a, iters, (int)nx, prow);
    return hipGetLastError() == hipSuccess ? VP2P_OK : VP2P_E_LAUNCH;
  };
  int g_first = 0;              // first CFG half / batch row the v1 kernel takes
  if constexpr (sizeof(T) == 2) {
    const bool p2p = a->prompts > 0 && a->batch == (a->cond_only ? 1 : 2) * a->prompts;
    const bool edit = p2p && (a->edit_mode != VP2P_EDIT_NONE || a->reweight);
    if (edit && !a->cond_only) {
      const int rc = launch_v3(0, a->prompts);     // the unconditional half: plain attention on v3
      if (rc != VP2P_OK) return rc;
      g_first = 1;
    }
    if (edit && a->prompts == 2) {
      const int rc = launch_v3e();
      if (rc == VP2P_OK) {
        if (a->lb_acc) {
          const int sets = a->lb_sets == 2 ? 2 : 1;
          const int64_t n = (int64_t)sets * a->prompts * FQ;
          const unsigned blocks = (unsigned)std::min<int64_t>((n + 255) / 256, 4096);
          hipLaunchKernelGGL(cross_lb_reduce_kernel, dim3(blocks), dim3(256), 0, s, a->lb_acc, a->lb_ws,
                             sets * a->prompts, a->heads, FQ);
          if (hipGetLastError() != hipSuccess) return VP2P_E_LAUNCH;
        }
        return VP2P_OK;
      }
      if (rc != VP2P_E_SHAPE) return rc;
    }
    if (!edit) {
      const int rc = launch_v3(0, a->batch);
      if (rc != VP2P_OK) return rc;
      const int sets = a->lb_sets == 2 ? 2 : 1;
      if (p2p && a->lb_acc) {
        const int64_t n = (int64_t)sets * a->prompts * FQ;
        const unsigned blocks = (unsigned)std::min<int64_t>((n + 255) / 256, 4096);
        hipLaunchKernelGGL(cross_lb_reduce_kernel, dim3(blocks), dim3(256), 0, s, a->lb_acc, a->lb_ws,
                           sets * a->prompts, a->heads, FQ);
        if (hipGetLastError() != hipSuccess) return VP2P_E_LAUNCH;
      }
      return VP2P_OK;
    }
  }
  const bool p2p = a->prompts > 0 && a->batch == (a->cond_only ? 1 : 2) * a->prompts;
  const int groups = (p2p ? (a->cond_only ? 1 : 2) : a->batch) - g_first;
  const int64_t items = (int64_t)((FQ + 31) / 32) * ((a->heads + 3) / 4);
  if (items <= 0 || groups > 65535) return VP2P_E_SHAPE;
  // One item per workgroup: measured faster at the UNet's shapes than a resident grid looping over
  // items with cross-item Q prefetch (res-64 d40: 113 vs 132 us, profiles/r01_k2_ab.txt); the loop
  // stays for grids beyond the 2^31 workgroup limit.
  const int64_t nwg = std::min<int64_t>(items, 0x7fffffff);
  const int prow = a->tokens_kv | 1;           // odd fp32 row stride: conflict-free per-lane rows
  const int rp = p2p ? a->prompts : 1;
  const int sets = a->lb_sets == 2 ? 2 : 1;
  const size_t lds = (size_t)4 * 32 * prow * sizeof(float) + (size_t)(rp - 1) * a->tokens_kv * 16 +
                     (size_t)sets * rp * a->tokens_kv * sizeof(float);
  hipLaunchKernelGGL((cross_attn_kernel<T, D, KB>), dim3((unsigned)nwg, (unsigned)groups), dim3(256), lds, s,
                     *a, prow, g_first);
  if (hipGetLastError() != hipSuccess) return VP2P_E_LAUNCH;
  if (p2p && a->lb_acc) {   // (set, prompt) pairs are contiguous: reduce them as sets*prompts rows
    const int64_t n = (int64_t)sets * a->prompts * FQ;
    const unsigned blocks = (unsigned)std::min<int64_t>((n + 255) / 256, 4096);
    hipLaunchKernelGGL(cross_lb_reduce_kernel, dim3(blocks), dim3(256), 0, s, a->lb_acc, a->lb_ws,
                       sets * a->prompts, a->heads, FQ);
    if (hipGetLastError() != hipSuccess) return VP2P_E_LAUNCH;
  }
  return VP2P_OK;
}

template <typename T, int D>
static int launch_cross_kb(const vp2p_cross_attn_args* a, hipStream_t s) {
  switch ((a->tokens_kv + 31) / 32) {
    case 1: return launch_cross<T, D, 1>(a, s);
    case 2: return launch_cross<T, D, 2>(a, s);
    case 3: return launch_cross<T, D, 3>(a, s);
    case 4: return launch_cross<T, D, 4>(a, s);
    default: return VP2P_E_SHAPE;
  }
}

template <typename T, int D>
static int launch_prep(const void* k, const void* v, int64_t k_sb, int64_t k_sn, int64_t v_sb,
                       int64_t v_sn, int batch, int nkv, int heads, void* ws, hipStream_t s) {
  using C = CrossCfg<T, D>;
  const int kp = 32 * ((nkv + 31) / 32);
  const int64_t total = cross_ws_elems<T>(batch, heads, kp, C::DP, C::DV);
  const int64_t blocks = std::min<int64_t>((total + 255) / 256, 4096);
  hipLaunchKernelGGL((cross_kv_prep_kernel<T, D>), dim3((unsigned)blocks), dim3(256), 0, s,
                     static_cast<const T*>(k), static_cast<const T*>(v), k_sb, k_sn, v_sb, v_sn,
                     batch, nkv, heads, kp, static_cast<T*>(ws));
  return hipGetLastError() == hipSuccess ? VP2P_OK : VP2P_E_LAUNCH;
}

}  // namespace vp2p

using namespace vp2p;

extern "C" int64_t vp2p_cross_kv_workspace_bytes(int32_t batch, int32_t tokens_kv, int32_t heads,
                                                 int32_t head_dim, int32_t dtype) {
  if (batch <= 0 || tokens_kv <= 0 || heads <= 0) return VP2P_E_ARG;
  if (tokens_kv > 128) return VP2P_E_SHAPE;
  if (dtype != VP2P_BF16 && dtype != VP2P_F32) return VP2P_E_DTYPE;
  int dp = 0, dv = 0;
  const int rc = cross_pad_dims(head_dim, dtype, dp, dv);
  if (rc) return rc;
  const int kp = 32 * ((tokens_kv + 31) / 32);
  return (int64_t)batch * heads * kp * (dp + dv) * (dtype == VP2P_BF16 ? 2 : 4);
}

extern "C" int vp2p_cross_kv_prep(const void* k, const void* v, int64_t k_sb, int64_t k_sn,
                                  int64_t v_sb, int64_t v_sn, int32_t batch, int32_t tokens_kv,
                                  int32_t heads, int32_t head_dim, int32_t dtype, void* kv_ws,
                                  void* stream) {
  if (!k || !v || !kv_ws || batch <= 0 || tokens_kv <= 0 || heads <= 0) return VP2P_E_ARG;
  if (tokens_kv > 128) return VP2P_E_SHAPE;
  hipStream_t s = static_cast<hipStream_t>(stream);
#define VP2P_PREP(DIM)                                                                          \
  case DIM:                                                                                      \
    return dtype == VP2P_BF16                                                                    \
               ? launch_prep<bf16, DIM>(k, v, k_sb, k_sn, v_sb, v_sn, batch, tokens_kv, heads, kv_ws, s) \
               : launch_prep<float, DIM>(k, v, k_sb, k_sn, v_sb, v_sn, batch, tokens_kv, heads, kv_ws, s);
  if (dtype != VP2P_BF16 && dtype != VP2P_F32) return VP2P_E_DTYPE;
  switch (head_dim) {
    VP2P_PREP(32) VP2P_PREP(40) VP2P_PREP(64) VP2P_PREP(80) VP2P_PREP(128) VP2P_PREP(160)
    default: return VP2P_E_HEAD_DIM;
  }
#undef VP2P_PREP
}

extern "C" int vp2p_cross_attn_p2p_fwd(const vp2p_cross_attn_args* a, void* stream) {
  if (!a || !a->q || !a->kv_ws || !a->o) return VP2P_E_ARG;
  if (a->batch <= 0 || a->frames <= 0 || a->tokens_q <= 0 || a->tokens_kv <= 0 || a->heads <= 0)
    return VP2P_E_ARG;
  if (a->tokens_kv > 128) return VP2P_E_SHAPE;
  const int esz = a->dtype == VP2P_BF16 ? 2 : (a->dtype == VP2P_F32 ? 4 : 0);
  if (!esz) return VP2P_E_DTYPE;
  const int epc = 16 / esz;
  const int64_t strides[] = {a->q_sb, a->q_sf, a->q_sn, a->o_sb, a->o_sf, a->o_sn};
  for (int64_t st : strides)
    if (st % epc) return VP2P_E_ARG;
  if (a->head_dim % epc || (reinterpret_cast<uintptr_t>(a->q) & 15) || (reinterpret_cast<uintptr_t>(a->o) & 15))
    return VP2P_E_ARG;
  if (a->cond_only && !(a->prompts > 0 && a->batch == a->prompts)) return VP2P_E_ARG;
  const bool p2p = a->prompts > 0 && a->batch == (a->cond_only ? 1 : 2) * a->prompts;
  if (p2p && a->prompts > 4) return VP2P_E_SHAPE;
  const bool edit = p2p && (a->edit_mode != VP2P_EDIT_NONE || a->reweight);
  if (edit) {
    if (!a->alpha_words) return VP2P_E_ARG;
    if (a->edit_mode == VP2P_EDIT_REPLACE && (!a->map_ptr || !a->map_idx || !a->map_val)) return VP2P_E_ARG;
    if (a->edit_mode == VP2P_EDIT_REFINE && (!a->map_idx || !a->refine_alpha)) return VP2P_E_ARG;
    if (a->reweight && !a->equalizer) return VP2P_E_ARG;
  }
  if (a->lb_acc && (!p2p || !a->lb_word_alpha || !a->lb_ws)) return VP2P_E_ARG;
  if (a->lb_sets < 0 || a->lb_sets > 2) return VP2P_E_ARG;
  hipStream_t s = static_cast<hipStream_t>(stream);
#define VP2P_CROSS(DIM) \
  case DIM: return a->dtype == VP2P_BF16 ? launch_cross_kb<bf16, DIM>(a, s) : launch_cross_kb<float, DIM>(a, s);
  switch (a->head_dim) {
    VP2P_CROSS(32) VP2P_CROSS(40) VP2P_CROSS(64) VP2P_CROSS(80) VP2P_CROSS(128) VP2P_CROSS(160)
    default: return VP2P_E_HEAD_DIM;
  }
#undef VP2P_CROSS
}
