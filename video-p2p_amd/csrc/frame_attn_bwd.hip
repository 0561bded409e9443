// K1b — backward of the shared-K/V attention: FrameAttention (tuneavideo/models/attention.py:282-322)
// and, with tokens_kv = 77, the plain hooked cross-attention (ptp_utils.py:206-220 under the
// DummyController, ptp_utils.py:225-234).  Needed by the null-text optimisation, which
// back-propagates the MSE of the DDIM step through the whole UNet to the unconditional embedding
// (run_videop2p.py:580-612, loss.backward() at :601).
//
// Math (S = scale * Q K^T, P = softmax(S), O = P V; dO given):
//   dV = P^T dO,  dP = dO V^T,  dS = P * (dP - delta),  delta_q = sum_d dO[q] O[q]
//   dQ = scale * dS K,  dK = scale * dS^T Q
// P is recomputed from the forward's row log-sum-exp (log2 units, vp2p_frame_attn_fwd .lse), so
// nothing of size queries x keys is ever stored.  dK/dV of a batch element sum over ALL its
// frames * tokens_q queries (every frame attends to the same keys).
//
// Two kernels, no float atomics:
//   dq  : query-parallel, like the forward: a wave owns 32 queries (query on the lane), streams the
//         K/V tiles through LDS; S^T = K Q^T and dP^T = V dO^T use the forward's swapped 32x32 MFMA
//         layout, dQ^T += K^T dS^T takes dS^T straight from the accumulator (K^T by transposed LDS
//         reads).  Also writes delta for the second kernel.
//   dkv : key-parallel: a wave owns 32 keys (key on the lane: K and V rows live in registers as the
//         B operands) and streams Q / dO tiles; S = Q K^T and dP = dO V^T land with the key on the
//         lane, so P and dS feed dV^T += dO^T P and dK^T += Q^T dS directly.  The query axis is
//         split over `splits` workgroups for parallelism; their fp32 partials are summed by a
//         third, elementwise kernel (skipped when splits == 1).
#include <stdlib.h>

#include "common.hpp"
#include "vp2p.h"

namespace vp2p {

template <typename T, int D>
struct BwdCfg {
  static constexpr bool BF = sizeof(T) == 2;
  static constexpr int KD = Mfma<T>::KD;
  static constexpr int DP = round_up(D, KD);     // K-dim of the Q.K^T-shaped products
  static constexpr int KS = DP / KD;
  static constexpr int DV = round_up(D, 32);     // M of the transposed-operand products
  static constexpr int NT = DV / 32;
  static constexpr int EPC = 16 / (int)sizeof(T);
  static constexpr int CPR = D / EPC;            // 16-byte chunks per row
  static constexpr int WIDTH = DP > DV ? DP : DV;
  // bf16: rows are read both with ds_read_b128 and ds_read_b64_tr_b16; the stride keeps the
  // transposed reads conflict-free (the row reads take a 4-way conflict).  f32: odd stride.
  static constexpr int row_bf16() {
    int v = WIDTH;
    while (!((v / 2) % 64 == 16 || (v / 2) % 64 == 48)) v += 8;
    return v;
  }
  static constexpr int ROW = BF ? row_bf16() : WIDTH + 1;
  static constexpr int TILE = 64;                // rows per staged LDS tile
  static constexpr int IMG = TILE * ROW;         // elements per image
  static constexpr int NCH = (TILE * CPR + 255) / 256;
};

// A operand = rows [row0, row0 + 32) of a row-major LDS image, Q.K^T k-step si.
template <typename T, int ROW>
__device__ __forceinline__ typename Mfma<T>::frag lds_row_frag(const T* img, int row0, int si) {
  const int l = lane_id(), r = l & 31, h = l >> 5;
  if constexpr (sizeof(T) == 2)
    return *reinterpret_cast<const bf16x8*>(img + (row0 + r) * ROW + 16 * si + 8 * h);
  else
    return img[(row0 + r) * ROW + 2 * si + h];
}

// A operand = transpose of the image: M = columns [32t, 32t + 32), K = rows row0.. in the
// accumulator's row order (so it pairs with Mfma<T>::p_frag of an accumulator tile), step sp.
template <typename T, int ROW>
__device__ __forceinline__ typename Mfma<T>::frag lds_tr_frag(const T* img, int row0, int sp, int t) {
  if constexpr (sizeof(T) == 2) {
    return vt_frag_lds<ROW>(img, row0, sp, t);
  } else {
    const int l = lane_id();
    return img[(row0 + f32_pv_key(sp, l >> 5)) * ROW + 32 * t + (l & 31)];
  }
}

// Stages TILE rows (16-byte chunks of D elements) into an LDS image: issue early, write late.
template <typename T, int D>
struct TileStage {
  using C = BwdCfg<T, D>;
  u32x4 reg[C::NCH];
  template <typename RowPtr>
  __device__ __forceinline__ void load(RowPtr rowptr) {
    const int tid = threadIdx.x;
#pragma unroll
    for (int i = 0; i < C::NCH; ++i) {
      const int c = tid + i * 256;
      const int row = c / C::CPR, col = (c - row * C::CPR) * C::EPC;
      const T* p = c < C::TILE * C::CPR ? rowptr(row) : nullptr;
      reg[i] = p ? *reinterpret_cast<const u32x4*>(p + col) : u32x4{0, 0, 0, 0};
    }
  }
  __device__ __forceinline__ void store(T* img) const {
    const int tid = threadIdx.x;
#pragma unroll
    for (int i = 0; i < C::NCH; ++i) {
      const int c = tid + i * 256;
      if (c < C::TILE * C::CPR) {
        const int row = c / C::CPR, col = (c - row * C::CPR) * C::EPC;
        if constexpr (C::BF) {
          *reinterpret_cast<u32x4*>(img + row * C::ROW + col) = reg[i];
        } else {
          float* d = reinterpret_cast<float*>(img) + row * C::ROW + col;
#pragma unroll
          for (int j = 0; j < 4; ++j) d[j] = __uint_as_float(reg[i][j]);
        }
      }
    }
  }
};

template <typename T>
__device__ __forceinline__ float frag_dot(typename Mfma<T>::frag a, typename Mfma<T>::frag b) {
  if constexpr (sizeof(T) == 2) {
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) s += (float)a[j] * (float)b[j];
    return s;
  } else {
    return a * b;
  }
}

// ---------------------------------------------------------------------------------------------
// dQ (+ delta).  Grid: batch * heads * ceil(FQ / 128), 4 waves x 32 queries.
// ---------------------------------------------------------------------------------------------
template <typename T, int D>
__global__ __launch_bounds__(256) void fa_bwd_dq_kernel(const vp2p_frame_attn_bwd_args a, float* delta) {
  using M = Mfma<T>;
  using C = BwdCfg<T, D>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  T* Ks = reinterpret_cast<T*>(smem);
  T* Vs = Ks + C::IMG;
  const int tid = threadIdx.x, l = tid & 63, w = tid >> 6, r = l & 31, h = l >> 5;
  const int FQ = a.frames * a.tokens_q, Nk = a.tokens_kv;
  const int qblocks = (FQ + 127) >> 7;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int bh = bid / qblocks, qb = bid - bh * qblocks;
  const int b = bh / a.heads, head = bh - b * a.heads;

  const int qi = qb * 128 + w * 32 + r;
  const bool qv = qi < FQ;
  const int fr = qv ? qi / a.tokens_q : 0, pos = qv ? qi - fr * a.tokens_q : 0;
  const int64_t qoff = (int64_t)b * a.q_sb + (int64_t)fr * a.q_sf + (int64_t)pos * a.q_sn + head * D;
  typename M::frag qf[C::KS], df[C::KS];
  float dl = 0.f;
#pragma unroll
  for (int s = 0; s < C::KS; ++s) {
    qf[s] = qv ? M::row_frag(static_cast<const T*>(a.q) + qoff, s, h, D) : M::zero();
    df[s] = qv ? M::row_frag(static_cast<const T*>(a.dout) + qoff, s, h, D) : M::zero();
    const typename M::frag of = qv ? M::row_frag(static_cast<const T*>(a.o) + qoff, s, h, D) : M::zero();
    dl += frag_dot<T>(df[s], of);
  }
  dl += xhalf(dl);
  const int64_t ridx = (int64_t)(b * a.heads + head) * FQ + qi;
  if (qv && h == 0) delta[ridx] = dl;
  const float lse = qv ? a.lse[ridx] : 0.f;
  const float cs = a.scale * kLog2e;

  for (int i = tid; i < 2 * C::IMG * (int)sizeof(T) / 16; i += 256)
    reinterpret_cast<u32x4*>(smem)[i] = u32x4{0, 0, 0, 0};

  const T* kbase = static_cast<const T*>(a.k) + (int64_t)b * a.kv_sb + head * D;
  const T* vbase = static_cast<const T*>(a.v) + (int64_t)b * a.kv_sb + head * D;
  TileStage<T, D> sk, sv;
  f32x16 dq[C::NT];
#pragma unroll
  for (int t = 0; t < C::NT; ++t) dq[t] = zero16();

  for (int kt = 0; kt < Nk; kt += C::TILE) {
    sk.load([&](int row) { return kt + row < Nk ? kbase + (int64_t)(kt + row) * a.kv_sn : nullptr; });
    sv.load([&](int row) { return kt + row < Nk ? vbase + (int64_t)(kt + row) * a.kv_sn : nullptr; });
    __syncthreads();
    sk.store(Ks);
    sv.store(Vs);
    __syncthreads();
#pragma unroll
    for (int key0 = 0; key0 < C::TILE; key0 += 32) {
      if (kt + key0 >= Nk) break;
      f32x16 s = zero16(), dp = zero16();
#pragma unroll
      for (int si = 0; si < C::KS; ++si) {
        s = M::mma(lds_row_frag<T, C::ROW>(Ks, key0, si), qf[si], s);
        dp = M::mma(lds_row_frag<T, C::ROW>(Vs, key0, si), df[si], dp);
      }
      f32x16 ds;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const bool kvld = kt + key0 + acc_row(i, h) < Nk;
        const float p = kvld ? fast_exp2(s[i] * cs - lse) : 0.f;
        ds[i] = p * (dp[i] - dl);
      }
#pragma unroll
      for (int sp = 0; sp < M::PV_STEPS; ++sp) {
        const typename M::frag bfr = M::p_frag(ds, sp);
#pragma unroll
        for (int t = 0; t < C::NT; ++t) dq[t] = M::mma(lds_tr_frag<T, C::ROW>(Ks, key0, sp, t), bfr, dq[t]);
      }
    }
  }
  if (qv) {
    T* orow = static_cast<T*>(a.dq) + qoff;
#pragma unroll
    for (int t = 0; t < C::NT; ++t)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int dc = 32 * t + 8 * g + 4 * h;
        if (dc < D) {
#pragma unroll
          for (int j = 0; j < 4; ++j) orow[dc + j] = M::from_f32(dq[t][4 * g + j] * a.scale);
        }
      }
  }
}

// ---------------------------------------------------------------------------------------------
// dK, dV.  Grid: batch * heads * splits * ceil(Nk / 128), 4 waves x 32 keys; split s covers
// query tiles [s * per, (s + 1) * per).
// ---------------------------------------------------------------------------------------------
template <typename T, int D>
__global__ __launch_bounds__(256) void fa_bwd_dkv_kernel(const vp2p_frame_attn_bwd_args a, const float* delta,
                                                         float* part, int splits) {
  using M = Mfma<T>;
  using C = BwdCfg<T, D>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  T* Qs = reinterpret_cast<T*>(smem);
  T* Os = Qs + C::IMG;                                        // dO image
  float* Ls = reinterpret_cast<float*>(Os + C::IMG);          // lse of the tile's queries (+inf past FQ)
  float* Ds = Ls + C::TILE;                                   // delta
  const int tid = threadIdx.x, l = tid & 63, w = tid >> 6, r = l & 31, h = l >> 5;
  const int FQ = a.frames * a.tokens_q, Nk = a.tokens_kv;
  const int kblocks = (Nk + 127) >> 7;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int kb = bid % kblocks;
  const int rest = bid / kblocks;
  const int sidx = rest % splits, bh = rest / splits;
  const int b = bh / a.heads, head = bh - b * a.heads;

  const int kj = kb * 128 + w * 32 + r;
  const bool kv = kj < Nk;
  const int64_t koff = (int64_t)b * a.kv_sb + (int64_t)kj * a.kv_sn + head * D;
  typename M::frag kf[C::KS], vf[C::KS];
#pragma unroll
  for (int s = 0; s < C::KS; ++s) {
    kf[s] = kv ? M::row_frag(static_cast<const T*>(a.k) + koff, s, h, D) : M::zero();
    vf[s] = kv ? M::row_frag(static_cast<const T*>(a.v) + koff, s, h, D) : M::zero();
  }
  for (int i = tid; i < 2 * C::IMG * (int)sizeof(T) / 16; i += 256)
    reinterpret_cast<u32x4*>(smem)[i] = u32x4{0, 0, 0, 0};

  const int qtiles = (FQ + C::TILE - 1) / C::TILE;
  const int per = (qtiles + splits - 1) / splits;
  const int qt0 = sidx * per, qt1 = min(qtiles, qt0 + per);
  const int64_t rbase = (int64_t)(b * a.heads + head) * FQ;
  const T* qb_ = static_cast<const T*>(a.q);
  const T* db_ = static_cast<const T*>(a.dout);
  auto qrow = [&](const T* base, int qi) -> const T* {
    if (qi >= FQ) return nullptr;
    const int fr = qi / a.tokens_q, pos = qi - fr * a.tokens_q;
    return base + (int64_t)b * a.q_sb + (int64_t)fr * a.q_sf + (int64_t)pos * a.q_sn + head * D;
  };
  const float cs = a.scale * kLog2e;
  TileStage<T, D> sq, so;
  f32x16 dk[C::NT], dv[C::NT];
#pragma unroll
  for (int t = 0; t < C::NT; ++t) dk[t] = dv[t] = zero16();

  for (int qt = qt0; qt < qt1; ++qt) {
    const int q00 = qt * C::TILE;
    sq.load([&](int row) { return qrow(qb_, q00 + row); });
    so.load([&](int row) { return qrow(db_, q00 + row); });
    float lv = 0.f, dv_ = 0.f;
    if (tid < C::TILE) {
      const int qi = q00 + tid;
      lv = qi < FQ ? a.lse[rbase + qi] : __builtin_huge_valf();
      dv_ = qi < FQ ? delta[rbase + qi] : 0.f;
    }
    __syncthreads();
    sq.store(Qs);
    so.store(Os);
    if (tid < C::TILE) {
      Ls[tid] = lv;
      Ds[tid] = dv_;
    }
    __syncthreads();
#pragma unroll
    for (int q0 = 0; q0 < C::TILE; q0 += 32) {
      if (q00 + q0 >= FQ) break;
      f32x16 s = zero16(), dp = zero16();
#pragma unroll
      for (int si = 0; si < C::KS; ++si) {
        s = M::mma(lds_row_frag<T, C::ROW>(Qs, q0, si), kf[si], s);
        dp = M::mma(lds_row_frag<T, C::ROW>(Os, q0, si), vf[si], dp);
      }
      f32x16 p, ds;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const f32x4 lq = *reinterpret_cast<const f32x4*>(Ls + q0 + 8 * g + 4 * h);
        const f32x4 dq = *reinterpret_cast<const f32x4*>(Ds + q0 + 8 * g + 4 * h);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float pv = fast_exp2(s[4 * g + j] * cs - lq[j]);
          p[4 * g + j] = pv;
          ds[4 * g + j] = pv * (dp[4 * g + j] - dq[j]);
        }
      }
#pragma unroll
      for (int sp = 0; sp < M::PV_STEPS; ++sp) {
        const typename M::frag pb = M::p_frag(p, sp), db = M::p_frag(ds, sp);
#pragma unroll
        for (int t = 0; t < C::NT; ++t) {
          dv[t] = M::mma(lds_tr_frag<T, C::ROW>(Os, q0, sp, t), pb, dv[t]);
          dk[t] = M::mma(lds_tr_frag<T, C::ROW>(Qs, q0, sp, t), db, dk[t]);
        }
      }
    }
    __syncthreads();
  }
  if (!kv) return;
  const int Cc = a.heads * D;
#pragma unroll
  for (int t = 0; t < C::NT; ++t)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int dc = 32 * t + 8 * g + 4 * h;
      if (dc < D) {
        if (splits == 1) {
          T* kd = static_cast<T*>(a.dk) + koff + dc;
          T* vd = static_cast<T*>(a.dv) + koff + dc;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            kd[j] = M::from_f32(dk[t][4 * g + j] * a.scale);
            vd[j] = M::from_f32(dv[t][4 * g + j]);
          }
        } else {
          float* pr = part + (((int64_t)sidx * a.batch + b) * Nk + kj) * 2 * Cc + head * D + dc;
          f32x4 k4, v4;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            k4[j] = dk[t][4 * g + j] * a.scale;
            v4[j] = dv[t][4 * g + j];
          }
          *reinterpret_cast<f32x4*>(pr) = k4;
          *reinterpret_cast<f32x4*>(pr + Cc) = v4;
        }
      }
    }
}

// Sums the split partials: (splits, batch, Nk, 2C) fp32 -> dk, dv (strided, dtype).  One thread per
// 4 channels.
template <typename T>
__global__ __launch_bounds__(256) void fa_bwd_reduce_kernel(const vp2p_frame_attn_bwd_args a, const float* part,
                                                            int splits) {
  const int Cc = a.heads * a.head_dim;
  const int64_t n4 = (int64_t)a.batch * a.tokens_kv * 2 * Cc / 4;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n4) return;
  const int64_t e = i * 4;
  const int c2 = (int)(e % (2 * Cc));
  const int64_t bk = e / (2 * Cc);
  const int key = (int)(bk % a.tokens_kv), b = (int)(bk / a.tokens_kv);
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  const int64_t stride = (int64_t)a.batch * a.tokens_kv * 2 * Cc;
  for (int s = 0; s < splits; ++s) acc += *reinterpret_cast<const f32x4*>(part + s * stride + e);
  const bool isv = c2 >= Cc;
  T* dst = static_cast<T*>(isv ? a.dv : a.dk) + (int64_t)b * a.kv_sb + (int64_t)key * a.kv_sn + (isv ? c2 - Cc : c2);
#pragma unroll
  for (int j = 0; j < 4; ++j) dst[j] = Mfma<T>::from_f32(acc[j]);
}

struct BwdPlan {
  int splits;
  int64_t delta_bytes, part_bytes;
};

static BwdPlan bwd_plan(const vp2p_frame_attn_bwd_args* a) {
  BwdPlan p;
  const int64_t FQ = (int64_t)a->frames * a->tokens_q;
  const int64_t kgroups = (int64_t)a->batch * a->heads * ((a->tokens_kv + 127) / 128);
  const int64_t qtiles = (FQ + 63) / 64;
  int64_t s = (1024 + kgroups - 1) / kgroups;
  s = s < qtiles / 4 ? s : qtiles / 4;   // >= 4 query tiles per split
  p.splits = (int)(s < 1 ? 1 : s);
  p.delta_bytes = round_up((int)0, 1) + ((int64_t)a->batch * a->heads * FQ * 4 + 255) / 256 * 256;
  p.part_bytes = p.splits > 1 ? (int64_t)p.splits * a->batch * a->tokens_kv * 2 * a->heads * a->head_dim * 4 : 0;
  return p;
}

template <typename T, int D>
static int launch_bwd(const vp2p_frame_attn_bwd_args* a, hipStream_t stream) {
  using C = BwdCfg<T, D>;
  const BwdPlan p = bwd_plan(a);
  float* delta = static_cast<float*>(a->workspace);
  float* part = reinterpret_cast<float*>(static_cast<char*>(a->workspace) + p.delta_bytes);
  const int64_t FQ = (int64_t)a->frames * a->tokens_q;
  const int64_t nq = (int64_t)a->batch * a->heads * ((FQ + 127) / 128);
  const int64_t nk = (int64_t)a->batch * a->heads * p.splits * ((a->tokens_kv + 127) / 128);
  if (nq > 0x7fffffff || nk > 0x7fffffff) return VP2P_E_SHAPE;
  const int lds_dq = 2 * C::IMG * (int)sizeof(T);
  const int lds_dkv = 2 * C::IMG * (int)sizeof(T) + 2 * C::TILE * 4;
  hipLaunchKernelGGL((fa_bwd_dq_kernel<T, D>), dim3((unsigned)nq), dim3(256), lds_dq, stream, *a, delta);
  hipLaunchKernelGGL((fa_bwd_dkv_kernel<T, D>), dim3((unsigned)nk), dim3(256), lds_dkv, stream, *a,
                     (const float*)delta, part, p.splits);
  if (p.splits > 1) {
    const int64_t n4 = (int64_t)a->batch * a->tokens_kv * 2 * a->heads * D / 4;
    hipLaunchKernelGGL((fa_bwd_reduce_kernel<T>), dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, stream, *a,
                       (const float*)part, p.splits);
  }
  return hipGetLastError() == hipSuccess ? VP2P_OK : VP2P_E_LAUNCH;
}

static int check_bwd(const vp2p_frame_attn_bwd_args* a) {
  if (!a || !a->q || !a->k || !a->v || !a->o || !a->dout || !a->lse || !a->dq || !a->dk || !a->dv ||
      !a->workspace)
    return VP2P_E_ARG;
  if (a->batch <= 0 || a->frames <= 0 || a->tokens_q <= 0 || a->tokens_kv <= 0 || a->heads <= 0 ||
      a->head_dim <= 0)
    return VP2P_E_ARG;
  const int esz = a->dtype == VP2P_BF16 ? 2 : (a->dtype == VP2P_F32 ? 4 : 0);
  if (!esz) return VP2P_E_DTYPE;
  const int epc = 16 / esz;
  const int64_t strides[] = {a->q_sb, a->q_sf, a->q_sn, a->kv_sb, a->kv_sn};
  for (int64_t s : strides)
    if (s % epc) return VP2P_E_ARG;
  const void* ptrs[] = {a->q, a->k, a->v, a->o, a->dout, a->dq, a->dk, a->dv, a->workspace};
  for (const void* p : ptrs)
    if (reinterpret_cast<uintptr_t>(p) & 15) return VP2P_E_ARG;
  if (a->head_dim % epc) return VP2P_E_ARG;
  return VP2P_OK;
}

}  // namespace vp2p

using namespace vp2p;

extern "C" int64_t vp2p_frame_attn_bwd_workspace_bytes(const vp2p_frame_attn_bwd_args* a) {
  if (!a || a->batch <= 0 || a->frames <= 0 || a->tokens_q <= 0 || a->tokens_kv <= 0 || a->heads <= 0 ||
      a->head_dim <= 0)
    return VP2P_E_ARG;
  const BwdPlan p = bwd_plan(a);
  return p.delta_bytes + p.part_bytes;
}

extern "C" int vp2p_frame_attn_bwd(const vp2p_frame_attn_bwd_args* a, void* stream) {
  const int st = check_bwd(a);
  if (st != VP2P_OK) return st;
  hipStream_t s = static_cast<hipStream_t>(stream);
#define VP2P_BWD_CASE(DIM) \
  case DIM:                \
    return a->dtype == VP2P_BF16 ? launch_bwd<bf16, DIM>(a, s) : launch_bwd<float, DIM>(a, s);
  switch (a->head_dim) {
    VP2P_BWD_CASE(32)
    VP2P_BWD_CASE(40)
    VP2P_BWD_CASE(64)
    VP2P_BWD_CASE(80)
    VP2P_BWD_CASE(128)
    VP2P_BWD_CASE(160)
    default:
      return VP2P_E_HEAD_DIM;
  }
#undef VP2P_BWD_CASE
}
