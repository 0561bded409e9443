// K1 at res-64 -- FrameAttention with first-frame K/V (tuneavideo/models/attention.py:282-322) in
// the form the UNet calls it there: bf16, head_dim 40, q pre-scaled by scale * log2(e) (the to_q
// GEMM's alpha), tokens_kv a multiple of 256 (other lengths: the x2f kernel).  These launches
// carry 88 % of K1's FLOPs.
//
// Why a separate kernel: at d = 40 a 32x32 score block is 7 MFMAs (3 QK^T k-steps, 4 PV) against
// 16 v_exp + 8 v_cvt per lane, so the SIMD's issue port -- not the matrix pipe -- is the tight
// resource, and the compiler-scheduled x2f loop (frame_attn.hip) keeps each block's exps waiting on
// that block's own QK^T MFMAs (its 8-exp bursts leave the matrix pipe idle).  Here one wave per SIMD
// runs SETS independent 32-query sets as one software pipeline over the whole key axis, with the
// instruction order written out slot by slot:
//  * an iteration (one 32-key block) is SETS groups of 7 MFMA slots; group g issues PV of set g's
//    previous block (4 MFMAs) and QK^T of the set whose exps the previous group finished (3 MFMAs),
//    and beside those 7 MFMAs the 16 v_exp + 8 v_cvt of set g: 2-3 exps and about one cvt per MFMA
//    gap (CDNA guide T19 / MI355X_MICROARCH 'vector-instruction ISSUE cost'), nothing waiting on an
//    MFMA of the same group;
//  * O^T lives in the accumulator file (AGPRs), written only by the PV MFMAs (inline asm, so hipcc
//    keeps it there); scores, P, Q and the K/V fragments fit the arch VGPRs;
//  * each K / V^T fragment is re-read as soon as its last MFMA of the block has issued, >= 5 MFMA
//    slots before its next use;
//  * K and V tiles of 256 keys arrive by LDS-DMA (buffer_load ... lds, 32-bit offsets, no register
//    staging) through a 3-slot ring with ONE barrier per tile: tile t+2 is issued right after tile
//    t's barrier, the first point where every wave is done with tile t-1;
//  * the LDS image of a tile is bank-conflict free for every fragment read (swz_* below): dims 0..31
//    of each key row as a 64-byte row whose four 16-byte chunks are XOR-swizzled by (row >> 2) & 3,
//    dims 32..39 as a separate 16-byte-row tail.  LDS-DMA writes each instruction's 64 chunks in lane
//    order, but which global chunk a lane fetches is free, so the permutation costs nothing.  (The
//    dense 80-byte rows it replaces put 2 of every 4-row ds_read_b64_tr_b16 group on one bank slot:
//    30 % of LDS-active cycles were conflicts, profiles/r04_k1_pp_pmc.txt.);
//  * the padding the MFMAs need is never stored: the K fragment of columns 40..47 (the folded -m
//    column: Q'[40] = -m, K[40] = 1) and V^T rows 40..63 (row 40 all ones = the row sum) are read by
//    the lanes that own them from a run of replicas of one 16-byte constant, laid so that the
//    fragment reads' immediate offsets land on one (broadcast reads, no per-read select);
//  * the row-sum growth check of x2f runs once per two tiles; when it moves m it also rescales the work
//    still in flight (every set's packed P, the next block's scores), so every term enters O at one
//    scale (CDNA guide T13 hazard).
#include "frame_attn.hpp"

// the product form: two 32-query sets per wave, two waves per SIMD (O in arch VGPRs, builtin MFMAs
// only); SETS 3 / WAVES 4 (one wave per SIMD, O in AGPRs) measured 0.85 vs 0.81 ms
#ifndef VP2P_K1_PP_SETS
#define VP2P_K1_PP_SETS 2
#endif
#ifndef VP2P_K1_PP_WAVES
#define VP2P_K1_PP_WAVES 8
#endif

namespace vp2p {

namespace {

typedef __attribute__((address_space(3))) char lchar;
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

// 256-key tiles: one barrier and one row-sum check per eight blocks; measured 0.7655 vs 0.780 ms
// (median) against 128-key tiles at res-64 B4 f8, same output (profiles/r04_k1_pp_kt256.jsonl)
// K fragments read this many blocks ahead (1: a group before their first use; 2 measured level,
// profiles/r05_k1_ab.jsonl)
#ifndef VP2P_K1_PP_KDIST
#define VP2P_K1_PP_KDIST 1
#endif
#ifndef VP2P_K1_PP_PIN
#define VP2P_K1_PP_PIN 1
#endif
// static priority for the second-dispatched half: 0.5-1 % (profiles/r05_k1_ab.jsonl)
#ifndef VP2P_K1_PP_PRIO
#define VP2P_K1_PP_PRIO 1
#endif
// lab-only timing diagnostics (wrong results): bit 0 no v_exp, 1 no K / V fragment reads in the
// loop, 2 no tile DMA in the loop, 3 no per-tile barrier, 4 no V^T reads, 5 no K reads
#ifndef VP2P_K1_DIAG
#define VP2P_K1_DIAG 0
#endif
#ifndef VP2P_K1_PP_KT
#define VP2P_K1_PP_KT 256
#endif
constexpr int kD = 40, kKT = VP2P_K1_PP_KT, kDiag = VP2P_K1_DIAG, KDIST = VP2P_K1_PP_KDIST;
constexpr int kNB = kKT / 32;                                      // 32-key blocks per tile
// a slot: main image [kKT][4 chunks] (dims 0..31), then the tail [kKT][1 chunk] (dims 32..39)
constexpr int kMainB = 64, kTailB = 16, kTail = kKT * kMainB;
constexpr int kSlotB = kKT * (kMainB + kTailB);                   // 20 KiB per K or V slot
constexpr int kNSlot = 3;
constexpr int kChunks = kKT * kD / 8;                             // 16-byte chunks per tile: 1280
constexpr int kDmaPerTile = kChunks / 64;                          // wave-instructions per tile: 20
static_assert(kChunks % 64 == 0 && kTail % 1024 == 0, "whole DMA instructions");
// LDS: K ring, V ring, then replicas [1, 0 x 7] in every 16-byte chunk of a run starting at bank
// slot 8 of a 256-B bank row (the V^T tail reads' constant lanes then never share a slot with
// their data lanes, which sit on slots 0..7 / 8..15 for the low / high rows: swz_* below)
constexpr int kKRing = 0, kVRing = kNSlot * kSlotB, kCR = 2 * kNSlot * kSlotB + 128;
constexpr int kRep = kKT + 1;                                     // reads land at kCR + 16 k, k <= kKT
constexpr int kLdsBytes = kCR + 16 * kRep;
static_assert((kCR / 16) % 16 == 8, "constant run on bank slot 8");
// the XOR swizzle of the main image: chunk c of key row r is stored at chunk 4 r + (c ^ swz(r))
__device__ __forceinline__ int swz(int r) { return (r >> 2) & 3; }

__device__ __forceinline__ bf16x8 ld128(const lchar* p) { return *reinterpret_cast<const __attribute__((address_space(3))) bf16x8*>(p); }
__device__ __forceinline__ bf16x4 ldtr(const lchar* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4bf16((__attribute__((address_space(3))) bf16x4*)(p));
}
// The inner loop is written out slot by slot: the MFMAs, v_exp and v_cvt of a slot are pinned to it
// by sched_barrier(0), and the scores are made opaque at every block start (an empty asm) so no IR
// pass hoists a block's exps into the previous one.  Only the LDS reads, their waits and the address
// arithmetic are placed by the compiler.  The one inline-asm MFMA (PV into AGPRs, one wave per SIMD)
// has hazards hipcc cannot see; the slot order excludes them:
//  * v_cvt -> PV MFMA reading the packed P: one whole block apart;
//  * VALU write of P / O in the rare rescale -> MFMA: the s_nop 1 opening every block;
//  * PV MFMA -> VALU read of O: o_fence() (two s_nop 7).
__device__ __forceinline__ uint32_t vcvt(float x, float y) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2){x, y}, bf16x2));
}
// S^T = K . Q'^T, three k-steps (builtins: hipcc pads their hazards, including those of any copy it
// makes of their operands)
__device__ __forceinline__ void qk_first(f32x16& acc, const bf16x8& k, const bf16x8& q) {
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(k, q, f32x16{}, 0, 0, 0);
}
__device__ __forceinline__ void qk_next(f32x16& acc, const bf16x8& k, const bf16x8& q) {
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(k, q, acc, 0, 0, 0);
}
__device__ __forceinline__ void sb() { __builtin_amdgcn_sched_barrier(0); }
// sched_barrier orders only what the instruction selector has chained (side effects): pure values --
// v_exp, v_cvt -- are linearised near their uses first, and a slot's exps / cvts whose scores came
// from an MFMA of the previous group sank past the group's MFMAs (the whole group's VALU after its
// last MFMA).  Passing each result through an empty volatile asm chains it to its slot.
#if VP2P_K1_PP_PIN
__device__ __forceinline__ void pin2(float& x, float& y) { asm volatile("" : "+v"(x), "+v"(y)); }
__device__ __forceinline__ uint32_t pin(uint32_t x) { asm volatile("" : "+v"(x)); return x; }
#else
__device__ __forceinline__ void pin2(float&, float&) {}
__device__ __forceinline__ uint32_t pin(uint32_t x) { return x; }
#endif

// O^T += V^T . P^T.  With one wave per SIMD O lives in the accumulator file (AGPRs) -- the arch
// VGPRs hold everything else -- which takes inline asm (hipcc picks the register file of a builtin's
// accumulator itself); with two waves per SIMD (256 registers per wave) everything, O included, fits
// the arch VGPRs and the builtin is used, so hipcc pads every hazard.
template <bool AGPR>
__device__ __forceinline__ void pv(f32x16& o, const bf16x8& v, const u32x4& p) {
  if constexpr (AGPR)
    asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(o) : "v"(v), "v"(__builtin_bit_cast(bf16x8, p)));
  else
    o = __builtin_amdgcn_mfma_f32_32x32x16_bf16(v, __builtin_bit_cast(bf16x8, p), o, 0, 0, 0);
}

}  // namespace

template <int SETS, int WAVES>
__global__ __launch_bounds__(64 * WAVES, WAVES / 4) void frame_attn_kernel_pp(const vp2p_frame_attn_args a) {
  static_assert(SETS >= 2, "the QK^T of the last set rides in group 0 of the next block");
  static_assert(WAVES == 4 || WAVES == 8, "one or two waves per SIMD");
  constexpr bool OA = WAVES == 4;                   // O in the accumulator file
  using T = bf16;
  using M = Mfma<T>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  lchar* const L = (lchar*)smem;

  const int tid = threadIdx.x, l = tid & 63, r = l & 31, h = l >> 5;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  constexpr int QW = 32 * SETS, QB = WAVES * QW;
  const int FQ = a.frames * a.tokens_q;
  const int qblocks = (FQ + QB - 1) / QB;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int bh = bid / qblocks, qb = bid - bh * qblocks;
  const int b = bh / a.heads, head = bh - b * a.heads;
  const int Nk = a.tokens_kv;
  const int ntiles = Nk / kKT;

  // queries: SETS sets of 32 per wave; Q'[40] (lane half 1, k-step 2, element 0) carries -m
  auto qrow_of = [&](int st, int& qi, int& fr, int& pos) {
    qi = qb * QB + w * QW + st * 32 + r;
    const bool v = qi < FQ;
    fr = v ? qi / a.tokens_q : 0;
    pos = v ? qi - fr * a.tokens_q : 0;
    return v;
  };
  bf16x8 qf[SETS][3];
#pragma unroll
  for (int st = 0; st < SETS; ++st) {
    int qi, fr, pos;
    const bool qv = qrow_of(st, qi, fr, pos);
    const T* qrow = static_cast<const T*>(a.q) + b * a.q_sb + fr * a.q_sf + pos * a.q_sn + head * kD;
#pragma unroll
    for (int s = 0; s < 3; ++s) qf[st][s] = qv ? M::row_frag(qrow, s, h, kD) : M::zero();
  }

  // K / V tile DMA: wave w issues instructions n = w, w + WAVES, ... (< 10) of each tile; lane l of
  // instruction n moves chunk 64n + l = (row, chunk-in-row) of the dense image
  const T* kb_ = static_cast<const T*>(a.k) + b * a.k_sb + head * kD;
  const T* vb_ = static_cast<const T*>(a.v) + b * a.v_sb + head * kD;
  const __amdgpu_buffer_rsrc_t krs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<T*>(kb_), 0, (uint32_t)((int64_t)(Nk - 1) * a.k_sn * 2 + kD * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t vrs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<T*>(vb_), 0, (uint32_t)((int64_t)(Nk - 1) * a.v_sn * 2 + kD * 2), 0x00020000);
  constexpr int NDMA = (kDmaPerTile + WAVES - 1) / WAVES;
  uint32_t kvo[NDMA], vvo[NDMA];
#pragma unroll
  for (int i = 0; i < NDMA; ++i) {
    // image chunk c: main (row c / 4, stored chunk c % 4 = source chunk (c % 4) ^ swz(row)) or tail
    const int c = 64 * (w + WAVES * i) + l;
    const bool main = c < kTail / 16;
    const int row = main ? c >> 2 : c - kTail / 16, ch = main ? (c & 3) ^ swz(c >> 2) : 4;
    kvo[i] = (uint32_t)(row * a.k_sn * 2 + ch * 16);
    vvo[i] = (uint32_t)(row * a.v_sn * 2 + ch * 16);
  }
  const uint32_t k_tile_b = (uint32_t)(kKT * a.k_sn * 2), v_tile_b = (uint32_t)(kKT * a.v_sn * 2);
  // The DMA is inline asm: hipcc would otherwise treat every later LDS read as dependent on it and
  // drain vmcnt to 0 before the first one.  M0 (the LDS destination) is an input operand ("{m0}"),
  // so hipcc sets it and knows it is live; the s_nop covers the M0 write -> LDS-DMA hazard.  Its completion is waited for explicitly (vmcnt(0) before
  // the barrier that publishes the tile).
  const uint32_t lds_base = (uint32_t)(uintptr_t)L;
  auto dma_tile = [&](int t) {
    const int tt = min(t, ntiles - 1);     // past the end: reload the last tile into a dead slot
    const int slot = t % kNSlot;
    const uint32_t ks = (uint32_t)tt * k_tile_b, vs = (uint32_t)tt * v_tile_b;
#pragma unroll
    for (int i = 0; i < NDMA; ++i) {
      const int n = w + WAVES * i;
      if (i + 1 < NDMA || n < kDmaPerTile) {
        const uint32_t kd = __builtin_amdgcn_readfirstlane(lds_base + kKRing + slot * kSlotB + n * 1024);
        const uint32_t vd = __builtin_amdgcn_readfirstlane(lds_base + kVRing + slot * kSlotB + n * 1024);
        asm volatile("s_nop 0\n\tbuffer_load_dwordx4 %0, %1, %3 offen lds"
                     :: "v"(kvo[i]), "s"(krs), "{m0}"(kd), "s"(ks) : "memory");
        asm volatile("s_nop 0\n\tbuffer_load_dwordx4 %0, %1, %3 offen lds"
                     :: "v"(vvo[i]), "s"(vrs), "{m0}"(vd), "s"(vs) : "memory");
      }
    }
  };

  // constant replicas, then tiles 0 and 1
  for (int i = tid; i < kRep; i += 64 * WAVES) {
    u32x4 c1 = {__builtin_bit_cast(uint16_t, (T)1.0f), 0u, 0u, 0u};
    *reinterpret_cast<__attribute__((address_space(3))) u32x4*>(L + kCR + 16 * i) = c1;
  }
  dma_tile(0);
  dma_tile(1);

  // per-lane LDS read offsets within a slot (the slot is added per tile; a block's key rows are
  // immediates: rows are 32-aligned, so swz() of a lane's row is fixed per lane).  Bank slots of the
  // reads (bank slot = 16-B chunk index mod 16; groups per MI355X_MICROARCH 'LDS'):
  //  K fragment, k-step s < 2: row r, chunk 2s + h -> slot 4 (r & 3) + ((2s + h) ^ swz(r)): each
  //    ds_read_b128 16-lane group holds rows {0-3,12-15,20-27} or {4-11,16-19,28-31}, whose swz()
  //    values are 0, 3, 1, 2 / 1, 2, 0, 3 per (r & 3): 16 distinct slots;
  //  K k-step 2: lane half 0 reads tail row r (slot r mod 16: distinct in each group), half 1 the
  //    fold constant (one address per instruction: a broadcast);
  const int k_s0 = r * kMainB + 16 * ((0 + h) ^ swz(r));
  const int k_s1 = r * kMainB + 16 * ((2 + h) ^ swz(r));
  const int k_t = kTail + r * kTailB;
  //  V^T fragment (vt_frag_lds geometry): lane (h, g, q, p) reads row 4h + q (+8 for the high half)
  //  of a 16-key step, columns 16g + 4p (dims 0..31: chunk 2g + p / 2 of the main image, swizzled by
  //  swz(row) = h (low) / h + 2 (high)); per 32-lane half the 4 rows x 4 chunks fill the 16 slots.
  //  Columns 32..39 (g = 0, p < 2) come from the tail (slots 4h + q / 8 + 4h + q), the rest of tile 1
  //  are the constant (slot 8 / 0: none of the data slots of the same read)
  const int vg = (l >> 4) & 1, q4 = (l >> 2) & 3, p4 = l & 3;
  const int v_lo = (4 * h + q4) * kMainB + 16 * ((2 * vg + (p4 >> 1)) ^ h) + 8 * (p4 & 1);
  const int v_hi = (8 + 4 * h + q4) * kMainB + 16 * ((2 * vg + (p4 >> 1)) ^ (h + 2)) + 8 * (p4 & 1);
  const int v_t = kTail + (4 * h + q4) * kTailB + 8 * (p4 & 1);
  const bool v1c = vg == 1 || p4 >= 2;
  const lchar* const v1const = L + kCR + ((vg == 0 && p4 == 2) ? 0 : 8);

  float m[SETS], lp[SETS];
  f32x16 o[SETS][2];
  f32x16 S[SETS];
  u32x4 P[SETS][2];
#pragma unroll
  for (int st = 0; st < SETS; ++st) {
    lp[st] = 0.f;
    o[st][0] = zero16();
    o[st][1] = zero16();
    P[st][0] = u32x4{0, 0, 0, 0};
    P[st][1] = u32x4{0, 0, 0, 0};
  }
  auto set_negm = [&](int st) {
    const bf16 nm = (bf16)(-m[st]);
    if (h == 1) qf[st][2][0] = nm;
  };

  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
#if VP2P_K1_PP_PRIO
  // static priority for the second-dispatched half (MI355X_MICROARCH 'Two waves per SIMD', item 4)
  if (w >= WAVES / 2) __builtin_amdgcn_s_setprio(1);
#endif

  // K fragments of the next KDIST blocks (kf[j % KDIST] = block j), V^T of the previous block
  bf16x8 kf[KDIST][3], vf[2][2];
  // m starts at the exact row max of keys 0..31 (fold slot still 0: S = q'.k)
  {
#pragma unroll
    for (int j = 0; j < KDIST; ++j) {
      kf[j][0] = ld128(L + kKRing + k_s0 + 32 * j * kMainB);
      kf[j][1] = ld128(L + kKRing + k_s1 + 32 * j * kMainB);
      kf[j][2] = ld128(h ? L + kCR : L + kKRing + k_t + 32 * j * kTailB);
    }
#pragma unroll
    for (int st = 0; st < SETS; ++st) {
      f32x16 s = M::mma(kf[0][0], qf[st][0], zero16());
      s = M::mma(kf[0][1], qf[st][1], s);
      s = M::mma(kf[0][2], qf[st][2], s);
      float v = s[0];
#pragma unroll
      for (int i = 1; i < 16; ++i) v = fmaxf(v, s[i]);
      m[st] = (float)(bf16)fmaxf(v, xhalf(v));
#pragma unroll
      for (int i = 0; i < 16; ++i) s[i] -= m[st];
      S[st] = s;
      set_negm(st);
    }
    // V "block -1" for the first PVs (P = 0: any finite data)
    const lchar* vb0 = L + kVRing + 16 * l;
#pragma unroll
    for (int sp = 0; sp < 2; ++sp)
#pragma unroll
      for (int t = 0; t < 2; ++t) vf[sp][t] = ld128(vb0);
  }

  // One block (iteration j).  On entry: S[g] = block j scores of sets 0..SETS-2 (at -m), S[SETS-1]
  // dead (its block j QK^T rides in group 0 here); P = block j-1 packed; kf = K block j; vf = V^T
  // block j-1.  Group 0 replaces kf by K block j+1 as its QK^T k-steps retire each fragment; the last
  // group replaces vf by V^T block j as its PVs retire each fragment.
  // kb0 / kb1: K k-step 0 / 1 bases, k2b: k-step 2 (tail or constant); vlo / vhi: V^T dims 0..31
  // of the low / high 8 rows, v1b: tile 1 (tail or constant)
  // j: the block's index in its tile (kf parity); krow: K rows of block j + KDIST from kb0 / kb1 / k2b
  auto block = [&](int j, const lchar* kb0, const lchar* kb1, const lchar* k2b, int krow, const lchar* vlo,
                   const lchar* vhi, const lchar* v1b, int vrow) {
    const int par = j % KDIST;
    sb();
    asm volatile("s_nop 1");
#pragma unroll
    for (int st = 0; st < SETS; ++st) asm volatile("" : "+v"(S[st]));
    auto v_tr = [&](int sp, int t) {
      const int rr = vrow + 16 * sp;
      const bf16x4 lo = t ? ldtr(v1b + rr * kTailB) : ldtr(vlo + rr * kMainB);
      const bf16x4 hi = t ? ldtr(v1b + rr * kTailB + 8 * kTailB) : ldtr(vhi + rr * kMainB);
      bf16x8 f;
#pragma unroll
      for (int j = 0; j < 4; ++j) { f[j] = lo[j]; f[4 + j] = hi[j]; }
      return f;
    };
#pragma unroll
    for (int g = 0; g < SETS; ++g) {
      const int qs = (g + SETS - 1) % SETS;                     // whose QK^T rides in this group
      const bool last = g == SETS - 1;
      float e[16];
      uint32_t pn[8];
      f32x16 acc;
      const f32x16& sg = S[g];
      // pair k = scores 2k, 2k+1.  (Moving some pairs onto a packed-f32 polynomial 2^x to unload the
      // transcendental unit measured slower, 0.92-1.02 vs 0.81 ms: the packed ops cost more issue
      // than the v_exp they replace -- profiles/r04_issue_bench.jsonl, r04_k1_poly_ab.jsonl.)
      auto pair = [&](int k) {
        e[2 * k] = (kDiag & 1) ? sg[2 * k] : fast_exp2(sg[2 * k]);
        e[2 * k + 1] = (kDiag & 1) ? sg[2 * k + 1] : fast_exp2(sg[2 * k + 1]);
        pin2(e[2 * k], e[2 * k + 1]);
      };
      // slot 0: pair 0 | QK k-step 0
      pair(0);
      // group 0: QK^T of the last set for block j (kf[par]), then kf[par] <- block j + KDIST;
      // the other groups: block j + 1
      bf16x8(&kg)[3] = kf[g == 0 ? par : (par + 1) % KDIST];
      qk_first(acc, kg[0], qf[qs][0]);
      if (g == 0 && !(kDiag & 34)) kg[0] = ld128(kb0 + krow * kMainB);
      sb();
      // slot 1: pair 1 | PV(sp 0, tile 1) | cvt pair 0
      pair(1);
      pv<OA>(o[g][1], vf[0][1], P[g][0]);
      pn[0] = pin(vcvt(e[0], e[1]));
      if (last && !(kDiag & 18)) vf[0][1] = v_tr(0, 1);
      sb();
      // slot 2: pair 2 | QK k-step 1 | cvt pair 1
      pair(2);
      qk_next(acc, kg[1], qf[qs][1]);
      pn[1] = pin(vcvt(e[2], e[3]));
      if (g == 0 && !(kDiag & 34)) kg[1] = ld128(kb1 + krow * kMainB);
      sb();
      // slot 3: pair 3 | PV(sp 0, tile 0) | cvt pair 2
      pair(3);
      pv<OA>(o[g][0], vf[0][0], P[g][0]);
      pn[2] = pin(vcvt(e[4], e[5]));
      if (last && !(kDiag & 18)) vf[0][0] = v_tr(0, 0);
      sb();
      // slot 4: pair 4 | QK k-step 2 -> S[qs] | cvt pair 3
      pair(4);
      qk_next(acc, kg[2], qf[qs][2]);
      pn[3] = pin(vcvt(e[6], e[7]));
      if (g == 0 && !(kDiag & 34)) kg[2] = ld128(k2b + krow * kTailB);
      sb();
      // slot 5: pair 5 | PV(sp 1, tile 1) | cvt pair 4
      pair(5);
      pv<OA>(o[g][1], vf[1][1], P[g][1]);
      pn[4] = pin(vcvt(e[8], e[9]));
      if (last && !(kDiag & 18)) vf[1][1] = v_tr(1, 1);
      sb();
      // slot 6: pairs 6-7 | PV(sp 1, tile 0) | cvt pairs 5-7
      pair(6);
      pair(7);
      pv<OA>(o[g][0], vf[1][0], P[g][1]);
      pn[5] = pin(vcvt(e[10], e[11]));
      pn[6] = pin(vcvt(e[12], e[13]));
      pn[7] = pin(vcvt(e[14], e[15]));
      if (last && !(kDiag & 18)) vf[1][0] = v_tr(1, 0);
      S[qs] = acc;
      P[g][0] = u32x4{pn[0], pn[1], pn[2], pn[3]};
      P[g][1] = u32x4{pn[4], pn[5], pn[6], pn[7]};
      sb();
    }
  };
  // O reads by the VALU: past the last PV MFMA's write (>= 12 wait states for this 8-pass MFMA)
  auto o_fence = [&]() {
#pragma unroll
    for (int st = 0; st < SETS; ++st)
      if constexpr (OA) asm volatile("s_nop 7\n\ts_nop 7" : "+a"(o[st][0]), "+a"(o[st][1]));
  };

  for (int t = 0; t < ntiles; ++t) {
    const int s0 = (t % kNSlot) * kSlotB, s1 = ((t + 1) % kNSlot) * kSlotB;
    // per-tile bases, opaque so hipcc folds the block offsets into the reads' immediates instead of
    // hoisting one address register per read out of the loop
    const lchar* ka0 = L + kKRing + s0 + k_s0;      // this tile's K
    const lchar* ka1 = L + kKRing + s0 + k_s1;
    const lchar* kn0 = L + kKRing + s1 + k_s0;      // the next tile's first block
    const lchar* kn1 = L + kKRing + s1 + k_s1;
    const lchar* vlo = L + kVRing + s0 + v_lo;
    const lchar* vhi = L + kVRing + s0 + v_hi;
    asm volatile("" : "+v"(ka0), "+v"(ka1), "+v"(kn0), "+v"(kn1), "+v"(vlo), "+v"(vhi));
    const lchar* k2a = h ? L + kCR : L + kKRing + s0 + k_t;
    const lchar* k2n = h ? L + kCR : L + kKRing + s1 + k_t;
    const lchar* v1b = v1c ? v1const : L + kVRing + s0 + v_t;
    asm volatile("" : "+v"(k2a), "+v"(k2n), "+v"(v1b));
    block(0, ka0, ka1, k2a, 32 * KDIST, vlo, vhi, v1b, 0);
    // tile t+1 (issued a tile ago) has landed; every wave is done with tile t-1's slot (K last read
    // in iteration kNB*t-2, V in kNB*t-1)
    if constexpr (!(kDiag & 8)) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
    if constexpr (!(kDiag & 4)) dma_tile(t + 2);
#pragma unroll
    for (int j = 1; j < kNB; ++j) {
      // block j + KDIST lies in this tile or (the last KDIST blocks) in the next one
      if (j + KDIST < kNB) block(j, ka0, ka1, k2a, 32 * (j + KDIST), vlo, vhi, v1b, 32 * j);
      else block(j, kn0, kn1, k2n, 32 * (j + KDIST - kNB), vlo, vhi, v1b, 32 * j);
    }
    // the row-sum growth check, at the end of every second tile (512 keys): 0.757-0.769 vs
    // 0.784-0.788 ms with one per tile, same output (profiles/r04_k1_pp_check_every.jsonl; one per
    // 1024 keys or none measured level with this).  Fewer checks only let p grow further before m
    // moves -- more range, the same relative precision; a row that overflows still ends in the exact
    // per-row fallback below.  At a check O holds blocks <= kNB(t+1)-2; P (block kNB(t+1)-1) and
    // S[0..SETS-2] (block kNB(t+1)) are still at the old m; S[SETS-1] is recomputed with the new fold.
    if ((t & 1) == 0) continue;
    sb();
    o_fence();
    float lc[SETS];
    bool grow = false;
#pragma unroll
    for (int st = 0; st < SETS; ++st) {
      lc[st] = o[st][1][4];             // O^T row 40 (lanes h == 0; the other half reads a zero row)
      grow |= lc[st] - lp[st] > kSumThr;
    }
    if (__any(grow)) {
#pragma unroll
      for (int st = 0; st < SETS; ++st) {
        const float mine = lc[st] - lp[st];
        const float other = xhalf(mine);
        const float dl = h == 0 ? mine : other;
        const float mn = dl > kSumThr ? (float)(bf16)(m[st] + __log2f(dl)) : m[st];
        const float alpha = fast_exp2(m[st] - mn);
        const float shift = m[st] - mn;
        m[st] = mn;
        set_negm(st);
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          o[st][0][i] *= alpha;
          o[st][1][i] *= alpha;
          S[st][i] += shift;
        }
        lc[st] *= alpha;
#pragma unroll
        for (int sp = 0; sp < 2; ++sp) {
          bf16x8 pp = __builtin_bit_cast(bf16x8, P[st][sp]);
#pragma unroll
          for (int j = 0; j < 8; ++j) pp[j] = (bf16)((float)pp[j] * alpha);
          P[st][sp] = __builtin_bit_cast(u32x4, pp);
        }
      }
    }
#pragma unroll
    for (int st = 0; st < SETS; ++st) lp[st] = lc[st];
  }
  // drain: PV of the last block
  sb();
  asm volatile("s_nop 1");
#pragma unroll
  for (int st = 0; st < SETS; ++st) {
    pv<OA>(o[st][1], vf[0][1], P[st][0]);
    pv<OA>(o[st][0], vf[0][0], P[st][0]);
    pv<OA>(o[st][1], vf[1][1], P[st][1]);
    pv<OA>(o[st][0], vf[1][0], P[st][1]);
  }
  o_fence();

#pragma unroll
  for (int st = 0; st < SETS; ++st) {
    int qi_, fr_, pos_;
    const bool qv_ = qrow_of(st, qi_, fr_, pos_);
    const float mine = o[st][1][4];
    const float other = xhalf(mine);
    const float lrow = h == 0 ? mine : other;
    bool bad = qv_ && (__float_as_uint(lrow) & 0x7f800000u) == 0x7f800000u;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int i = 0; i < 16; ++i) bad |= qv_ && (__float_as_uint(o[st][t][i]) & 0x7f800000u) == 0x7f800000u;
    if (qv_ && !bad) {
      if (a.lse) a.lse[(int64_t)(b * a.heads + head) * FQ + qi_] = m[st] + log2f(lrow);
      const float inv = 1.f / lrow;
      T* orow = static_cast<T*>(a.o) + b * a.o_sb + fr_ * a.o_sf + pos_ * a.o_sn + head * kD;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int gg = 0; gg < 4; ++gg) {
          const int dc = 32 * t + 8 * gg + 4 * h;
          if (dc < kD) {
            bf16x4 v;
#pragma unroll
            for (int j = 0; j < 4; ++j) v[j] = (bf16)(o[st][t][4 * gg + j] * inv);
            *reinterpret_cast<bf16x4*>(orow + dc) = v;
          }
        }
    }
    if (bad) frame_attn_exact_row<kD>(a, b, head, fr_, pos_, qi_, h, 1.f);
  }
}

int launch_frame_attn_pp(const vp2p_frame_attn_args* a, hipStream_t stream) {
  constexpr int SETS = VP2P_K1_PP_SETS, WAVES = VP2P_K1_PP_WAVES;
  if (a->dtype != VP2P_BF16 || a->head_dim != kD || !a->q_prescaled || a->tokens_kv % kKT) return VP2P_E_SHAPE;
  // 32-bit buffer offsets: every key row of one (b, head) within 4 GiB
  if ((int64_t)a->tokens_kv * a->k_sn * 2 >= (1ll << 32) || (int64_t)a->tokens_kv * a->v_sn * 2 >= (1ll << 32))
    return VP2P_E_SHAPE;
  const int FQ = a->frames * a->tokens_q;
  const int64_t nwg = (int64_t)a->batch * a->heads * ((FQ + 32 * SETS * WAVES - 1) / (32 * SETS * WAVES));
  if (nwg <= 0 || nwg > 0x7fffffff) return VP2P_E_SHAPE;
  static const bool attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&frame_attn_kernel_pp<SETS, WAVES>),
                                               hipFuncAttributeMaxDynamicSharedMemorySize, kLdsBytes) == hipSuccess;
  if (!attr) return VP2P_E_LAUNCH;
  hipLaunchKernelGGL((frame_attn_kernel_pp<SETS, WAVES>), dim3((unsigned)nwg), dim3(64 * WAVES), kLdsBytes, stream, *a);
  return hipGetLastError() == hipSuccess ? VP2P_OK : VP2P_E_LAUNCH;
}

}  // namespace vp2p
