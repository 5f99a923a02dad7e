// A12 Miller loops in two passes (pairing.hpp "Two-pass Miller loop"):
//   k_miller_lines: one lane per DISTINCT message: T walks the 68 steps over Q = H(m); each step's Q-only
//                   line (l0, c1, c4) goes to HBM, SoA limb-major (step s, word w of message u at
//                   lines[(s * W_LINE + w) * nm + u]: coalesced).  Lines depend on H(m) only, so every set
//                   and unit signing the same root shares them;
//   k_miller_acc:   one lane per chunk of <= K pairings of one batch group: f = prod_s prod_items line_s(P)
//                   with shared squarings, from the stored lines; writes conj(f).  An item is either one set
//                   (P = r_i pk_i) or, with same-message merging, a unit: the included sets of one batch
//                   group that sign the same root (P = sum r_i pk_i; the pairing is bilinear, so
//                   prod_i e(r_i pk_i, H(m)) = e(sum_i r_i pk_i, H(m))).
//   k_miller_acc2:  the same accumulation on TWO lanes per chunk, each holding half of f (no spills): the default
//                   for one-item chunks (runs below 131,072 pairings); chunks of >= 2 stay on one lane (faster).
//   k_miller_lines2 (lane pairs, fp2x.hpp) and k_miller_coop (one 192-lane workgroup per pairing, small runs).
// Line traffic is 68 x 84 words = 22.8 KB per message (HBM-cheap next to ~5,200 Montgomery products).
#include "k_common.hpp"
#include "gt_wave.hpp"
#include "gt6.hpp"
#include "gtx.hpp"

// Line pairs in the one-lane chunk loop (line_pair + fp12_mul_by_line2: 23 Fp2 products per two items instead of 26):
// correct (test_line_pair_product, chunk-form GPU parity) but the pending line and the denser product raise the
// kernel's scratch 480 -> 1,600 B/lane, and the driver's C2 measured 3.03M vs 3.06M without (r4zn): off.
#ifndef BLS_LINE_PAIRS
#define BLS_LINE_PAIRS 0
#endif
// Line pairs in the two-lane accumulation: the pair's line product split three and three over the lanes, then each
// lane one half of f times it (6 + 5 Fp2 products): 14 products per lane per two items instead of 16.  Correct (the
// chunk-form parity tests pass with it) but the pending line and M spill (1,280 B/lane): forced two-lane chunks of
// two measured 2.92M vs 3.47M for the default one-lane form (100 steps): off.
#ifndef BLS_ACC2_PAIRS
#define BLS_ACC2_PAIRS 0
#endif

BLS_INL fp fp_add_n(const fp& a, const fp& b) { return fp_add_norm(a, b); }

// LDS-staged line prefetch for the accumulation kernels (north star: "LDS staging of precomputed line coefficients").
// The accumulation runs one wave per SIMD, so nothing hides the HBM latency of the 84 line words an item needs at each
// step (SQ: 19-22% of its wave-cycles waiting).  Each lane's next line (the next item of the step, or the chunk's first
// item of the next step) is fetched straight into LDS by global_load_lds_dword -- no VGPRs held while it is in flight
// -- as soon as the current one has been read out, so it arrives during the current item's sparse product (or the
// next step's squaring).  Word-major slot: word w of lane t at pre[w * WAVE + t] (the DMA writes lane t's dword at
// M0 + 4 t); one slot per one-wave workgroup, 21.5 KB.  Measured (round 6, profiles/r06_lds_prefetch_ab.json): parity
// green, no gain (C2 3.27M vs 3.30M at 20 steps, 3.81M vs 3.82M at 100; the Miller stage no faster) -- the waiting is
// not the line loads -- so off by default.
#ifndef BLS_ACC_PREFETCH
#define BLS_ACC_PREFETCH 0
#endif
#if BLS_ACC_PREFETCH && defined(__HIP_DEVICE_COMPILE__)
#define LDS_AS __attribute__((address_space(3)))
// a rolled loop over the 84 words: one running address (the unrolled form kept 84 64-bit addresses live and spilled)
__device__ __forceinline__ void line_prefetch(uint32_t* pre, const uint32_t* o, uint32_t nm, uint32_t m) {
  const uint32_t* a = o + opaque_u32(m);
#pragma unroll 1
  for (int w = 0; w < W_LINE; w++) {
    __builtin_amdgcn_global_load_lds((const void*)a, (LDS_AS void*)(pre + w * WAVE), 4, 0, 0);
    a += nm;
  }
}
// the prefetched line is in LDS (vmcnt(0): global_load_lds completes through the vector memory counter)
__device__ __forceinline__ void line_wait() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_waitcnt(0x0F70);
  asm volatile("" ::: "memory");
}
// the slot's words are in registers (lgkmcnt(0)) before the next prefetch may overwrite it
__device__ __forceinline__ void line_read_done() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_waitcnt(0xC07F);
  asm volatile("" ::: "memory");
}
__device__ __forceinline__ fp ld_fp_pre(const uint32_t* pre, int w0) {
  fp r;
#pragma unroll
  for (int l = 0; l < BLS_NL; l++) r.l[l] = pre[(w0 + l) * WAVE + threadIdx.x];
  return r;
}
__device__ __forceinline__ fp2 ld_fp2_pre(const uint32_t* pre, int w0) {
  return fp2_make(ld_fp_pre(pre, w0), ld_fp_pre(pre, w0 + W_FP));
}
#define ACC_PREFETCH 1
#else
#define ACC_PREFETCH 0
#endif

STAGE_KERNEL_W(BLSGPU_WPE_LINES) void k_miller_lines(PipelineBuffers b) {
  uint32_t u = blockIdx.x * WAVE + threadIdx.x;
  if (u >= b.n_umsg || (b.mflags[u] & MF_H_INF)) return;
  miller_lines_store(ld_g2a(b.h_aff, b.nm, u), b.lines, b.nm, u);
}

// The same lines on lane pairs (fp2x.hpp): lane 2u + k holds coefficient k of T's coordinates and stores coefficient
// k of each line element -- half the per-lane state, two waves per SIMD.  Q is re-read at the five addition steps.
#ifndef BLSGPU_WPE_LINES2
#define BLSGPU_WPE_LINES2 2
#endif
STAGE_KERNEL_W(BLSGPU_WPE_LINES2) void k_miller_lines2(PipelineBuffers b) {
  const uint32_t q = blockIdx.x * WAVE + threadIdx.x;
  const uint32_t u = q >> 1, k = q & 1;
  if (u >= b.n_umsg || (b.mflags[u] & MF_H_INF)) return;  // both lanes of a pair leave together
  auto ldQ = [&] {
    const uint32_t uu = opaque_u32(u);
    aff<fp2x> Q;
    Q.x.v = ld_fp(b.h_aff, b.nm, uu, (int)(k * W_FP));
    Q.y.v = ld_fp(b.h_aff, b.nm, uu, (int)((2 + k) * W_FP));
    return Q;
  };
  g2projx Tp;
  {
    const aff<fp2x> Q = ldQ();
    Tp.x = Q.x;
    Tp.y = Q.y;
    Tp.z = F_one((const fp2x*)0);
  }
  int bit = 62;
  bool add_next = false;
#pragma unroll 1
  for (int s = 0; s < MILLER_STEPS; s++) {
    line3x Ln;
    if (!add_next) {
      miller_dbl_line(Tp, Ln);
      add_next = (BLS_Z_ABS >> bit) & 1ull;
      bit--;
    } else {
      miller_add_line(Tp, ldQ(), Ln);
      add_next = false;
    }
    uint32_t* o = b.lines + (size_t)s * W_LINE * b.nm;
    st_fp(o, b.nm, u, (int)(k * W_FP), Ln.l0.v);
    st_fp(o, b.nm, u, (int)((2 + k) * W_FP), Ln.c1.v);
    st_fp(o, b.nm, u, (int)((4 + k) * W_FP), Ln.c4.v);
  }
}

// One lane per chunk: f = prod over the chunk's items of f_{|z|,Q_item}(P_item), with ONE Fp12 squaring per
// doubling step for the whole chunk (the multi-pairing form of blst's miller_loop_n): K items cost
// 63 squarings + 68 K line multiplications instead of K (63 + 68).  UNITS: item u is pairing unit u
// (P = unit_p[u]); otherwise item i is a set (P = r_i pk_i, only if it enters the batch equation).
template <bool UNITS>
STAGE_KERNEL_W(BLSGPU_WPE_ACC) void k_miller_acc(PipelineBuffers b) {
  const uint32_t c = blockIdx.x * WAVE + threadIdx.x;
  if (c >= b.n_chunks) return;
  const uint32_t k0 = b.chunk_first[c], k1 = b.chunk_first[c + 1];
#if ACC_PREFETCH
  __shared__ uint32_t pre[W_LINE * WAVE];
  auto msg_of = [&](uint32_t k) {
    const uint32_t i = b.chunk_items[k];
    return UNITS ? b.unit_msg[i] : b.msg_idx[i];
  };
  if (k1 > k0) line_prefetch(pre, b.lines, b.nm, msg_of(k0));
#endif
  fp12 f = fp12_one();
  int bit = 62;
  bool add_next = false;
#pragma unroll 1
  for (int s = 0; s < MILLER_STEPS; s++) {
    if (!add_next && s != 0) f = fp12_sqr(f);
    const uint32_t* o = b.lines + (size_t)s * W_LINE * b.nm;
#if BLS_LINE_PAIRS
    // the chunk's lines two at a time: their product first (line_pair, 6 Fp2 products), then f times it (17) -- 23
    // products per two items against 26 for two sparse products
    bool pend = false;
    fp2 q0, q1, q4;
#endif
#pragma unroll 1
    for (uint32_t k = k0; k < k1; k++) {
      const uint32_t i = b.chunk_items[k];
      uint32_t m;
      bool active;
      if (UNITS) {
        m = b.unit_msg[i];
        active = b.unit_ok[i] != 0;
      } else {
        m = b.msg_idx[i];
        active = b.include[i] != 0;
      }
#if ACC_PREFETCH
      // this item's line (fetched into the slot one item ahead), then the slot takes the next one
      line_wait();
      line3 L;
      L.l0 = ld_fp2_pre(pre, 0);
      L.c1 = ld_fp2_pre(pre, 2 * W_FP);
      L.c4 = ld_fp2_pre(pre, 4 * W_FP);
      line_read_done();
      if (k + 1 < k1)
        line_prefetch(pre, o, b.nm, msg_of(k + 1));
      else if (s + 1 < MILLER_STEPS)
        line_prefetch(pre, o + (size_t)W_LINE * b.nm, b.nm, msg_of(k0));
      if (!active || (b.mflags[m] & MF_H_INF)) continue;
      const g1a P = ld_g1a(UNITS ? b.unit_p : b.pk_aff, b.n, i);
#else
      if (!active || (b.mflags[m] & MF_H_INF)) continue;
      const g1a P = ld_g1a(UNITS ? b.unit_p : b.pk_aff, b.n, i);
      line3 L;
      L.l0 = ld_fp2(o, b.nm, m, 0);
      L.c1 = ld_fp2(o, b.nm, m, 2 * W_FP);
      L.c4 = ld_fp2(o, b.nm, m, 4 * W_FP);
#endif
#if BLS_LINE_PAIRS
      const fp2 l1 = fp2_mul_fp(L.c1, P.x), l4 = fp2_mul_fp(L.c4, P.y);
      if (pend) {
        f = fp12_mul_by_line2(f, line_pair(q0, q1, q4, L.l0, l1, l4));
        pend = false;
      } else {
        q0 = L.l0;
        q1 = l1;
        q4 = l4;
        pend = true;
      }
#else
      f = fp12_mul_by_014(f, L.l0, fp2_mul_fp(L.c1, P.x), fp2_mul_fp(L.c4, P.y));
#endif
    }
#if BLS_LINE_PAIRS
    if (pend) f = fp12_mul_by_014(f, q0, q1, q4);
#endif
    if (!add_next) {
      add_next = (BLS_Z_ABS >> bit) & 1ull;
      bit--;
    } else {
      add_next = false;
    }
  }
  st_fp12(b.f_chunk, b.n, c, fp12_conj(f));
}

// Mid-size runs (latency with the chip not filled by one lane per pairing): TWO lanes per pairing, lane h of the
// pair holding half c_h of f = c0 + c1 w (Fp6 each) and the partner's half arriving by a lane exchange (__shfl_xor,
// no LDS).  Per step each lane does one Fp6 product of the complex squaring (lane 0: t = c0 c1, lane 1:
// s = (c0 + c1)(c0 + v c1); then c1' = 2t, c0' = s - t - v t) and one half of the sparse line product
// (c0' = c0 L01 + v (c1 l4 v), c1' = c1 L01 + c0 (l4 v)): 14 Fp2 products per lane per step against 25 on one lane, so
// a pairing takes ~0.56 of the lane-per-pairing time (12% more work in all).  A chunk of K items shares the squaring
// (one per step, split as above) and takes each item's sparse product on the two halves: f's 168 words never sit on
// one lane, so the kernel runs without spills (the one-lane chunk form spilled ~100 KB of scratch traffic per pairing).
template <bool UNITS>
STAGE_KERNEL_W(BLSGPU_WPE_ACC) void k_miller_acc2(PipelineBuffers b) {
  const uint32_t q = blockIdx.x * WAVE + threadIdx.x;
  const uint32_t c = q >> 1, h = q & 1;  // both lanes of a pair see the same c (WAVE is even)
  if (c >= b.n_chunks) return;           // whole pairs leave together: the exchanges below stay within live pairs
  const uint32_t k0 = b.chunk_first[c], k1 = b.chunk_first[c + 1];
#if ACC_PREFETCH
  __shared__ uint32_t pre[W_LINE * WAVE];
  auto msg_of = [&](uint32_t k) {
    const uint32_t i = b.chunk_items[k];
    return UNITS ? b.unit_msg[i] : b.msg_idx[i];
  };
  if (k1 > k0) line_prefetch(pre, b.lines, b.nm, msg_of(k0));
#endif
  fp6 mine = h ? fp6_zero() : fp6_one();
  int bit = 62;
  bool add_next = false;
#pragma unroll 1
  for (int s = 0; s < MILLER_STEPS; s++) {
    if (!add_next && s != 0) {
      const fp6 other = fp6_xlane(mine);
      const fp6 a0 = h ? other : mine, a1 = h ? mine : other;
      fp6 X, Y;  // lane 0: (a0, a1); lane 1: (a0 + a1, a0 + v a1), normalized, values <= 4p (fp6_mul's contract)
      if (h) {
        X.c0 = fp2_make(fp_add_n(a0.c0.c0, a1.c0.c0), fp_add_n(a0.c0.c1, a1.c0.c1));
        X.c1 = fp2_make(fp_add_n(a0.c1.c0, a1.c1.c0), fp_add_n(a0.c1.c1, a1.c1.c1));
        X.c2 = fp2_make(fp_add_n(a0.c2.c0, a1.c2.c0), fp_add_n(a0.c2.c1, a1.c2.c1));
        Y.c0 = fp2_make(fp_lc(T<1>(a0.c0.c0), T<1>(a1.c2.c0), T<-1>(a1.c2.c1)),
                        fp_lc(T<1>(a0.c0.c1), T<1>(a1.c2.c0), T<1>(a1.c2.c1)));
        Y.c1 = fp2_make(fp_add_n(a0.c1.c0, a1.c0.c0), fp_add_n(a0.c1.c1, a1.c0.c1));
        Y.c2 = fp2_make(fp_add_n(a0.c2.c0, a1.c1.c0), fp_add_n(a0.c2.c1, a1.c1.c1));
      } else {
        X = a0;
        Y = a1;
      }
      const fp6 pr = fp6_mul(X, Y);
      const fp6 t = fp6_xlane(pr);  // lane 1 receives t = a0 a1
      fp6 r;
      if (h) {  // c0' = s - t - v t, v t = (xi t2, t0, t1)
        r.c0.c0 = fp_lc(T<1>(pr.c0.c0), T<-1>(t.c0.c0), T<-1>(t.c2.c0), T<1>(t.c2.c1));
        r.c0.c1 = fp_lc(T<1>(pr.c0.c1), T<-1>(t.c0.c1), T<-1>(t.c2.c0), T<-1>(t.c2.c1));
        r.c1.c0 = fp_lc(T<1>(pr.c1.c0), T<-1>(t.c1.c0), T<-1>(t.c0.c0));
        r.c1.c1 = fp_lc(T<1>(pr.c1.c1), T<-1>(t.c1.c1), T<-1>(t.c0.c1));
        r.c2.c0 = fp_lc(T<1>(pr.c2.c0), T<-1>(t.c2.c0), T<-1>(t.c1.c0));
        r.c2.c1 = fp_lc(T<1>(pr.c2.c1), T<-1>(t.c2.c1), T<-1>(t.c1.c1));
      } else {  // c1' = 2t
        r.c0 = fp2_make(fp_lc(T<2>(pr.c0.c0)), fp_lc(T<2>(pr.c0.c1)));
        r.c1 = fp2_make(fp_lc(T<2>(pr.c1.c0)), fp_lc(T<2>(pr.c1.c1)));
        r.c2 = fp2_make(fp_lc(T<2>(pr.c2.c0)), fp_lc(T<2>(pr.c2.c1)));
      }
      mine = fp6_xlane(r);  // lane 0 computed c1', lane 1 c0': swap back
    }
    const uint32_t* o = b.lines + (size_t)s * W_LINE * b.nm;
    // mine <- mine-half of f * (T0 + T1 w) given T0 = mine x M0-part, T1 = other x M1-part: lane 0 c0' = T0 + v T1,
    // lane 1 c1' = T0 + T1
    auto fold = [&](const fp6& T0, const fp6& T1) {
      const fp6 T1v = h ? T1 : fp6_mul_v(T1);
      fp6 r;
      r.c0 = fp2_make(fp_lc(T<1>(T0.c0.c0), T<1>(T1v.c0.c0)), fp_lc(T<1>(T0.c0.c1), T<1>(T1v.c0.c1)));
      r.c1 = fp2_make(fp_lc(T<1>(T0.c1.c0), T<1>(T1v.c1.c0)), fp_lc(T<1>(T0.c1.c1), T<1>(T1v.c1.c1)));
      r.c2 = fp2_make(fp_lc(T<1>(T0.c2.c0), T<1>(T1v.c2.c0)), fp_lc(T<1>(T0.c2.c1), T<1>(T1v.c2.c1)));
      mine = r;
    };
#if BLS_ACC2_PAIRS
    bool pend = false;
    fp2 q0, q1, q4;
#endif
#pragma unroll 1
    for (uint32_t k = k0; k < k1; k++) {
      const uint32_t i = b.chunk_items[k];
      uint32_t m;
      bool active;
      if (UNITS) {
        m = b.unit_msg[i];
        active = b.unit_ok[i] != 0;
      } else {
        m = b.msg_idx[i];
        active = b.include[i] != 0;
      }
#if ACC_PREFETCH
      line_wait();
      fp2 l0 = ld_fp2_pre(pre, 0), l1 = ld_fp2_pre(pre, 2 * W_FP), l4 = ld_fp2_pre(pre, 4 * W_FP);
      line_read_done();
      if (k + 1 < k1)
        line_prefetch(pre, o, b.nm, msg_of(k + 1));
      else if (s + 1 < MILLER_STEPS)
        line_prefetch(pre, o + (size_t)W_LINE * b.nm, b.nm, msg_of(k0));
      if (!active || (b.mflags[m] & MF_H_INF)) continue;  // the same on both lanes of the pair
      const g1a P = ld_g1a(UNITS ? b.unit_p : b.pk_aff, b.n, i);
      l1 = fp2_mul_fp(l1, P.x);
      l4 = fp2_mul_fp(l4, P.y);
#else
      if (!active || (b.mflags[m] & MF_H_INF)) continue;  // the same on both lanes of the pair
      const g1a P = ld_g1a(UNITS ? b.unit_p : b.pk_aff, b.n, i);
      const fp2 l0 = ld_fp2(o, b.nm, m, 0);
      const fp2 l1 = fp2_mul_fp(ld_fp2(o, b.nm, m, 2 * W_FP), P.x);
      const fp2 l4 = fp2_mul_fp(ld_fp2(o, b.nm, m, 4 * W_FP), P.y);
#endif
#if BLS_ACC2_PAIRS
      if (!pend) {
        q0 = l0;
        q1 = l1;
        q4 = l4;
        pend = true;
        continue;
      }
      pend = false;
      // the two lines' product (tower.hpp line_pair) split over the pair: lane 0 P00, P11, X01, lane 1 P44, X04, X14
      const fp2 R1 = fp2_mul(h ? q4 : q0, h ? l4 : l0);
      const fp2 R2 = fp2_mul(h ? fp2_add_nr(q0, q4) : q1, h ? fp2_add_nr(l0, l4) : l1);
      const fp2 R3 = fp2_mul(h ? fp2_add_nr(q1, q4) : fp2_add_nr(q0, q1), h ? fp2_add_nr(l1, l4) : fp2_add_nr(l0, l1));
      const fp2 O1 = fp2_xlane(R1), O2 = fp2_xlane(R2), O3 = fp2_xlane(R3);
      const fp2 P00 = h ? O1 : R1, P44 = h ? R1 : O1, P11 = h ? O2 : R2, X04 = h ? R2 : O2, X01 = h ? O3 : R3,
                X14 = h ? R3 : O3;
      fp6 M0;
      M0.c0 = fp2_make(fp_lc(T<1>(P00.c0), T<1>(P44.c0), T<-1>(P44.c1)), fp_lc(T<1>(P00.c1), T<1>(P44.c0), T<1>(P44.c1)));
      M0.c1 = F2_LC3(X01, P00, P11);
      M0.c2 = P11;
      const fp2 m11 = F2_LC3(X04, P00, P44), m12 = F2_LC3(X14, P11, P44);
      // f * M (M1 = (0, m11, m12)): lane 0 c0' = f0 M0 + v f1 M1, lane 1 c1' = f1 M0 + f0 M1
      const fp6 other = fp6_xlane(mine);
      fold(fp6_mul(mine, M0), fp6_mul_by_12(other, m11, m12));
#else
      // lane 0: c0' = c0 (l0 + l1 v) + v (c1 (l4 v)); lane 1: c1' = c1 (l0 + l1 v) + c0 (l4 v)
      const fp6 other = fp6_xlane(mine);
      fold(fp6_mul_by_01(mine, l0, l1), fp6_mul_by_1(other, l4));
#endif
    }
#if BLS_ACC2_PAIRS
    if (pend) {  // an odd item: its sparse product alone
      const fp6 other = fp6_xlane(mine);
      fold(fp6_mul_by_01(mine, q0, q1), fp6_mul_by_1(other, q4));
    }
#endif
    if (!add_next) {
      add_next = (BLS_Z_ABS >> bit) & 1ull;
      bit--;
    } else {
      add_next = false;
    }
  }
  // f_chunk[c] = conj(f) = (c0, -c1): lane h writes its half (words 6 h W_FP .. )
  const fp6 out = h ? fp6_neg(mine) : mine;
  st_fp2(b.f_chunk, b.n, c, 6 * (int)h * W_FP, out.c0);
  st_fp2(b.f_chunk, b.n, c, (6 * (int)h + 2) * W_FP, out.c1);
  st_fp2(b.f_chunk, b.n, c, (6 * (int)h + 4) * W_FP, out.c2);
}

// The accumulation on lane pairs (gtx.hpp): lane 2c + k holds coefficient k of every Fp2 coefficient of chunk c's f
// (84 registers), so the kernel runs two waves per SIMD; the same chunks as k_miller_acc (K items sharing each
// squaring), the same work per pairing (25 Fp2 products per doubling step for one-item chunks, 12 / K + 13 for K),
// each Fp2 product split as two 588-MAD halves.  Each lane loads its coefficients of the lines and scales them by P.
#ifndef BLSGPU_WPE_ACCX
#define BLSGPU_WPE_ACCX 2
#endif
template <bool UNITS>
STAGE_KERNEL_W(BLSGPU_WPE_ACCX) void k_miller_accx(PipelineBuffers b) {
  const uint32_t q = blockIdx.x * WAVE + threadIdx.x;
  const uint32_t c = q >> 1, k = q & 1;
  if (c >= b.n_chunks) return;  // whole pairs leave together
  const uint32_t k0 = b.chunk_first[c], k1 = b.chunk_first[c + 1];
  fp12x f;
  f.c0.c0 = F_one((const fp2x*)0);
  f.c0.c1 = f.c0.c2 = f.c1.c0 = f.c1.c1 = f.c1.c2 = F_zero((const fp2x*)0);
  int bit = 62;
  bool add_next = false;
#pragma unroll 1
  for (int s = 0; s < MILLER_STEPS; s++) {
    if (!add_next && s != 0) f = fp12x_sqr(f);
    const uint32_t* o = b.lines + (size_t)s * W_LINE * b.nm;
#pragma unroll 1
    for (uint32_t it = k0; it < k1; it++) {
      const uint32_t i = b.chunk_items[it];
      uint32_t m;
      bool active;
      if (UNITS) {
        m = b.unit_msg[i];
        active = b.unit_ok[i] != 0;
      } else {
        m = b.msg_idx[i];
        active = b.include[i] != 0;
      }
      if (!active || (b.mflags[m] & MF_H_INF)) continue;  // the same on both lanes of the pair
      const g1a P = ld_g1a(UNITS ? b.unit_p : b.pk_aff, b.n, i);
      const fp2x l0{ld_fp(o, b.nm, m, (int)(k * W_FP))};
      const fp2x l1{fp_mul(ld_fp(o, b.nm, m, (int)((2 + k) * W_FP)), P.x)};
      const fp2x l4{fp_mul(ld_fp(o, b.nm, m, (int)((4 + k) * W_FP)), P.y)};
      f = fp12x_mul_by_014(f, l0, l1, l4);
    }
    if (!add_next) {
      add_next = (BLS_Z_ABS >> bit) & 1ull;
      bit--;
    } else {
      add_next = false;
    }
  }
  // f_chunk[c] = conj(f) = (c0, -c1): lane k writes coefficient k of the six slots
  st_fp(b.f_chunk, b.n, c, (int)((0 + k) * W_FP), f.c0.c0.v);
  st_fp(b.f_chunk, b.n, c, (int)((2 + k) * W_FP), f.c0.c1.v);
  st_fp(b.f_chunk, b.n, c, (int)((4 + k) * W_FP), f.c0.c2.v);
  st_fp(b.f_chunk, b.n, c, (int)((6 + k) * W_FP), fp_neg(f.c1.c0.v));
  st_fp(b.f_chunk, b.n, c, (int)((8 + k) * W_FP), fp_neg(f.c1.c1.v));
  st_fp(b.f_chunk, b.n, c, (int)((10 + k) * W_FP), fp_neg(f.c1.c2.v));
}

// Mid-size runs (latency): SIX lanes per pairing, lane k of a group holding the w-basis coefficient f_k of
// f = sum_k f_k w^k (w^6 = xi; tower slots c0.c0, c1.c0, c0.c1, c1.c1, c0.c2, c1.c2), ten groups per wave.  Every lane
// runs ONE instruction stream (no divergence inside a group): per step
//   square:  g_k = sum over i + j = k (mod 6) of f_i f_j (xi where i + j >= 6) -- 21 Fp2 products spread as 4 product
//            slots per lane (lane-dependent operands from a packed table, one operand doubled for the cross terms, the
//            xi twist applied by selects inside the lazily reduced recombination; the odd lanes' 4th slot is empty);
//   line:    h_k = g_k L0 + g_{k-2} L2 + g_{k-3} L3 (xi where the index wraps), L2 = c1 xP, L3 = c4 yP formed one Fp
//            product per lane (lanes 0-3) and gathered;
// operands move between the lanes of a group by ds_bpermute (__shfl).  ~7 Fp2 products per lane per doubling step
// against 14 in the two-lane form: the accumulation of a 2k-16k-pairing run (one wave per SIMD, 10,922 pairings per
// 1,024 waves) in about half the two-lane time, at ~1.7x the one-lane form's total work.
// WPE: waves per SIMD the kernel is compiled for -- 1 (301 registers, no scratch) for runs whose groups fit one wave
// per SIMD, 2 (256 registers, 192 B of scratch) above that (r05: 16k calls 12.9 -> 12.4 ms, 4k calls 9.3 -> 10.5 ms)
template <bool UNITS, int WPE>
__global__ __launch_bounds__(WAVE) __attribute__((amdgpu_waves_per_eu(WPE, WPE))) void k_miller_acc6(PipelineBuffers b) {
  const uint32_t lane = threadIdx.x, grp = lane / 6, k = lane % 6;
  const uint32_t c = blockIdx.x * ACC6_GROUPS + grp;
  if (grp >= ACC6_GROUPS || c >= b.n_chunks) return;  // whole groups leave together
  const int base = (int)(grp * 6);
  const uint32_t k0 = b.chunk_first[c], k1 = b.chunk_first[c + 1];
  fp2 f = k == 0 ? fp2_one() : fp2_zero();
  int bit = 62;
  bool add_next = false;
#pragma unroll 1
  for (int s = 0; s < MILLER_STEPS; s++) {
    if (!add_next && s != 0) {
      f = g6_sqr(f, G6{base, k});
    }
    const uint32_t* o = b.lines + (size_t)s * W_LINE * b.nm;
#pragma unroll 1
    for (uint32_t it = k0; it < k1; it++) {
      const uint32_t i = b.chunk_items[it];
      uint32_t m;
      bool active;
      if (UNITS) {
        m = b.unit_msg[i];
        active = b.unit_ok[i] != 0;
      } else {
        m = b.msg_idx[i];
        active = b.include[i] != 0;
      }
      if (!active || (b.mflags[m] & MF_H_INF)) continue;  // the same on every lane of the group
      const g1a Pa = ld_g1a(UNITS ? b.unit_p : b.pk_aff, b.n, i);
      f = g6_line_mul(f, o, b.nm, m, Pa.x, Pa.y, G6{base, k});
    }
    if (!add_next) {
      add_next = (BLS_Z_ABS >> bit) & 1ull;
      bit--;
    } else {
      add_next = false;
    }
  }
  // f_chunk[c] = conj(f): coefficient k -> tower slot (k odd: c1, else c0) . (k / 2), odd coefficients negated
  const int slot = (k & 1 ? 3 : 0) + (int)(k >> 1);
  st_fp2(b.f_chunk, b.n, c, slot * 2 * W_FP, (k & 1) ? fp2_neg(f) : f);
}

// Small runs (latency): one 128-lane workgroup per pairing, the Miller loop as cooperative Fp12 arithmetic
// (gt_wave.hpp: lines computed on the fly, one Fp product per lane per step) -- the same value as
// k_miller_lines + k_miller_acc with one item per chunk, in ~1/6 of the time per pairing, at a fraction of the
// lanes' efficiency; the runtime uses it only when the run's pairings fit the chip (runtime.cpp kCoopMaxItems).
template <bool UNITS>
__global__ __launch_bounds__(GTW_MILLER_LANES) void k_miller_coop(PipelineBuffers b) {
  __shared__ GtwLds sh;
  const uint32_t c = blockIdx.x, t = threadIdx.x;
  if (c >= b.n_chunks) return;
  const uint32_t i = b.chunk_items[b.chunk_first[c]];  // one item per chunk
  uint32_t m;
  bool active;
  if (UNITS) {
    m = b.unit_msg[i];
    active = b.unit_ok[i] != 0;
  } else {
    m = b.msg_idx[i];
    active = b.include[i] != 0;
  }
  active = active && !(b.mflags[m] & MF_H_INF);  // uniform over the workgroup
  if (active) {
    if (t < 4) lds_st(sh.QA, (int)t, ld_fp(b.h_aff, b.nm, m, (int)t * W_FP));
    const g1a P = ld_g1a(UNITS ? b.unit_p : b.pk_aff, b.n, i);
    gtw_sync();
    gtw_miller_loop(sh.G, sh.QA, P.x, P.y, sh.TB, sh.L, sh.L1, sh.S, sh.S2, t);
  } else {
    gtw_set_one(sh.G, t);
  }
  gtw_sync();
  for (uint32_t w = t; w < W_FP12; w += GTW_MILLER_LANES) b.f_chunk[(size_t)w * b.n + c] = sh.G[gtw_lds_word(w)];
}

static inline dim3 grid_for(uint32_t n) { return dim3((n + WAVE - 1) / WAVE); }

void launch_miller_coop(const PipelineBuffers& b, bool units, hipStream_t s, bool exclusive) {
  if (!b.n_chunks) return;
  if (units)
    hipLaunchKernelGGL(k_miller_coop<true>, dim3(b.n_chunks), dim3(GTW_MILLER_LANES),
                       exclusive ? exclusive_cu_lds<k_miller_coop<true>>() : 0, s, b);
  else
    hipLaunchKernelGGL(k_miller_coop<false>, dim3(b.n_chunks), dim3(GTW_MILLER_LANES),
                       exclusive ? exclusive_cu_lds<k_miller_coop<false>>() : 0, s, b);
}

void launch_miller_lines(const PipelineBuffers& b, hipStream_t s) {
  if (b.n_umsg) hipLaunchKernelGGL(k_miller_lines, grid_for(b.n_umsg), dim3(WAVE), 0, s, b);
}
void launch_miller_lines2(const PipelineBuffers& b, hipStream_t s) {
  if (b.n_umsg) hipLaunchKernelGGL(k_miller_lines2, grid_for(2 * b.n_umsg), dim3(WAVE), 0, s, b);
}
void launch_miller_acc2(const PipelineBuffers& b, bool units, hipStream_t s) {
  if (!b.n_chunks) return;
  if (units)
    hipLaunchKernelGGL(k_miller_acc2<true>, grid_for(2 * b.n_chunks), dim3(WAVE), 0, s, b);
  else
    hipLaunchKernelGGL(k_miller_acc2<false>, grid_for(2 * b.n_chunks), dim3(WAVE), 0, s, b);
}
// one wave per SIMD while the groups fit in 1,024 waves (256 CUs x 4 SIMDs), else two
#define ACC6_W1_MAX_CHUNKS (1024 * ACC6_GROUPS)
void launch_miller_acc6(const PipelineBuffers& b, bool units, hipStream_t s) {
  if (!b.n_chunks) return;
  const dim3 grid((b.n_chunks + ACC6_GROUPS - 1) / ACC6_GROUPS);
  const bool w2 = b.n_chunks > ACC6_W1_MAX_CHUNKS;
  if (units && w2)
    hipLaunchKernelGGL((k_miller_acc6<true, 2>), grid, dim3(WAVE), 0, s, b);
  else if (units)
    hipLaunchKernelGGL((k_miller_acc6<true, 1>), grid, dim3(WAVE), 0, s, b);
  else if (w2)
    hipLaunchKernelGGL((k_miller_acc6<false, 2>), grid, dim3(WAVE), 0, s, b);
  else
    hipLaunchKernelGGL((k_miller_acc6<false, 1>), grid, dim3(WAVE), 0, s, b);
}
void launch_miller_accx(const PipelineBuffers& b, bool units, hipStream_t s) {
  if (!b.n_chunks) return;
  if (units)
    hipLaunchKernelGGL(k_miller_accx<true>, grid_for(2 * b.n_chunks), dim3(WAVE), 0, s, b);
  else
    hipLaunchKernelGGL(k_miller_accx<false>, grid_for(2 * b.n_chunks), dim3(WAVE), 0, s, b);
}
void launch_miller_acc(const PipelineBuffers& b, bool units, hipStream_t s) {
  if (!b.n_chunks) return;
  if (units)
    hipLaunchKernelGGL(k_miller_acc<true>, grid_for(b.n_chunks), dim3(WAVE), 0, s, b);
  else
    hipLaunchKernelGGL(k_miller_acc<false>, grid_for(b.n_chunks), dim3(WAVE), 0, s, b);
}
