// TEST HARNESS ONLY: compiles the per-element device logic (lodestar_amd/csrc/*.hpp) for the host CPU
// so tests can check the exact kernel arithmetic against the oracle without a GPU.  It is never linked
// into libblsgpu.so (the product has no CPU path).  Byte formats: canonical big-endian 48-byte Fp.
#include <string.h>
#include "../../lodestar_amd/csrc/ops.hpp"
#include "../../lodestar_amd/csrc/msm.hpp"
#include "../../lodestar_amd/csrc/lacc.hpp"
#include "../../lodestar_amd/csrc/g2_coop.hpp"
#include "../../lodestar_amd/csrc/gt_wave.hpp"

#if defined(BLS_COUNT_OPS)
unsigned long long bls_count_mul = 0, bls_count_sqr = 0, bls_count_half = 0;
#endif

static fp load_mont(const uint8_t* b) {
  fp x;
  fp_from_be48_plain(b, x, 0xff);
  return fp_to_mont(x);
}
static fp2 load2(const uint8_t* b) { return fp2_make(load_mont(b + 48), load_mont(b)); }  // c1||c0
static void store2(const fp2& a, uint8_t* b) {
  fp_to_be48(a.c1, b);
  fp_to_be48(a.c0, b + 48);
}
static g2a load_g2(const uint8_t* b) {
  g2a p;
  p.x = load2(b);
  p.y = load2(b + 96);
  return p;
}
static g1a load_g1(const uint8_t* b) {
  g1a p;
  p.x = load_mont(b);
  p.y = load_mont(b + 48);
  return p;
}
// Fp12 -> 12 x 48 bytes, tower order c0.c0.c0, c0.c0.c1, c0.c1.c0, ... c1.c2.c1
static void store12(const fp12& f, uint8_t* b) {
  const fp6* s[2] = {&f.c0, &f.c1};
  int k = 0;
  for (int i = 0; i < 2; i++) {
    const fp2* t[3] = {&s[i]->c0, &s[i]->c1, &s[i]->c2};
    for (int j = 0; j < 3; j++) {
      fp_to_be48(t[j]->c0, b + 48 * k++);
      fp_to_be48(t[j]->c1, b + 48 * k++);
    }
  }
}
static fp12 load12(const uint8_t* b) {
  fp12 f;
  fp6* s[2] = {&f.c0, &f.c1};
  int k = 0;
  for (int i = 0; i < 2; i++) {
    fp2* t[3] = {&s[i]->c0, &s[i]->c1, &s[i]->c2};
    for (int j = 0; j < 3; j++) {
      t[j]->c0 = load_mont(b + 48 * k++);
      t[j]->c1 = load_mont(b + 48 * k++);
    }
  }
  return f;
}

// the device's regular signed-window scalar multiplication (k_common.hpp jac_mul_scalar_word: r = a + b lambda,
// Straus over the two 8-digit halves), host table
template <class F>
static jac<F> emu_mul_scalar_word(const jac<F>& P, uint64_t w) {
  jac<F> tab[8];
  const jac<F> P2 = jac_dbl(P);
  tab[0] = P;
  for (int e = 1; e < 8; e++) tab[e] = jac_add(tab[e - 1], P2);
  auto pick = [&](int k, bool hi) {
    const int d = 2 * (int)((w >> (4 * (hi ? k + 8 : k))) & 15u) - 15;
    jac<F> q = tab[(d < 0 ? -d : d) >> 1];
    if (hi) q = endo_lambda(q);
    return d < 0 ? jac_neg(q) : q;
  };
  jac<F> r = jac_add(pick(7, false), pick(7, true));
  for (int k = 6; k >= 0; k--)
    r = jac_add(jac_add(jac_dbl(jac_dbl(jac_dbl(jac_dbl(r)))), pick(k, false)), pick(k, true));
  return r;
}
// The bucket MSM of k_msm.hip (msm.hpp) over n affine points with scalar words w: buckets filled in set order
// (the kernel's list order), then the window sums and the Horner pass.  `active[i] == 0` skips point i.
static g2j emu_msm_core(const g2a* P, const uint64_t* w, const uint8_t* active, int n) {
  static g2j B[MSM_WINDOWS][MSM_BUCKETS];
  for (int k = 0; k < MSM_WINDOWS; k++)
    for (int e = 0; e < MSM_BUCKETS; e++) B[k][e] = jac_infinity<fp2>();
  for (int i = 0; i < n; i++) {
    if (active && !active[i]) continue;
    for (int k = 0; k < MSM_WINDOWS; k++) {
      bool neg;
      const uint32_t e = msm_bucket(w[i], k, neg);
      if (e == MSM_NO_BUCKET) continue;
      g2a q = P[i];
      if (neg) q.y = fp2_neg(q.y);
      B[k][e] = jac_add_aff(B[k][e], q);
    }
  }
  static g2j W[MSM_WINDOWS];
  for (int k = 0; k < MSM_WINDOWS; k++) W[k] = msm_window_sum_tree([&](int e) { return B[k][e]; });
  return msm_horner([&](int k) { return W[k]; });
}
extern "C" {
// sum_i r_i P_i through the bucket MSM; returns 0 for the point at infinity
int emu_msm(const uint8_t* pts192, const uint64_t* w, const uint8_t* active, int n, uint8_t* out192) {
  static g2a P[4096];
  if (n > 4096) return -1;
  for (int i = 0; i < n; i++) P[i] = load_g2(pts192 + 192 * (size_t)i);
  g2a a;
  if (!jac_to_aff(emu_msm_core(P, w, active, n), a)) return 0;
  g2a_to_be192(a, out192);
  return 1;
}
// the batch-scalar multiplications themselves (r = a + b lambda of word w; word 0 = the digits' value too)
int emu_g1_mul_word(const uint8_t* pk96, uint64_t w, uint8_t* out96) {
  g1a a;
  if (!jac_to_aff(emu_mul_scalar_word(jac_from_aff(load_g1(pk96)), w), a)) return 0;
  g1a_to_be96(a, out96);
  return 1;
}
int emu_g2_mul_word(const uint8_t* sig192, uint64_t w, uint8_t* out192) {
  g2a a;
  if (!jac_to_aff(emu_mul_scalar_word(jac_from_aff(load_g2(sig192)), w), a)) return 0;
  g2a_to_be192(a, out192);
  return 1;
}
// lacc_fin on raw limb sums (14 + 14 words), raw limbs out
void emu_lacc_fin(const uint32_t* pos, const uint32_t* neg, uint32_t* out14) {
  lacc a;
  for (int i = 0; i < BLS_NL; i++) {
    a.pos[i] = pos[i];
    a.neg[i] = neg[i];
  }
  const fp r = lacc_fin(a);
  for (int i = 0; i < BLS_NL; i++) out14[i] = r.l[i];
}
// the cooperative squaring's lazy operands: Mont((x0 + x1) (x0 - x1)) with x0 - x1 as fp_sub_k8, raw limbs in / out
void emu_sqr_operands_mul(const uint32_t* x0, const uint32_t* x1, uint32_t* out14) {
  fp a, b;
  for (int i = 0; i < BLS_NL; i++) {
    a.l[i] = x0[i];
    b.l[i] = x1[i];
  }
  const fp r = fp_mul(fp_add_nr(a, b), fp_sub_k8(a, b));
  for (int i = 0; i < BLS_NL; i++) out14[i] = r.l[i];
}
// the cooperative doubling chain (g2_coop.hpp, phases run lane by lane): [|z|]P for an affine P
int emu_g2c_mul_zabs(const uint8_t* p192, uint8_t* out192) {
  const g2a a = load_g2(p192);
  const g2j r = g2c_host_mul_zabs(jac_from_aff(a), [&] { return jac_from_aff(a); });
  g2a o;
  if (!jac_to_aff(r, o)) return 0;
  g2a_to_be192(o, out192);
  return 1;
}
// the cooperative addition (g2_coop.hpp g2c_add, phases lane by lane) of P and Q given affine (or infinity), each
// lifted to Jacobian coordinates with a different Z; returns 0 for the point at infinity
static g2j emu_lift(const g2a& a, int inf, uint32_t k) {
  if (inf) return jac_infinity<fp2>();
  fp zc0 = fp_zero(), zc1 = fp_one();
  zc0.l[0] = k;  // Z = k + u (Montgomery limbs: any nonzero value will do)
  const fp2 z = fp2_make(zc0, zc1), z2 = fp2_sqr(z);
  g2j r;
  r.x = fp2_mul(a.x, z2);
  r.y = fp2_mul(a.y, fp2_mul(z2, z));
  r.z = z;
  return r;
}
int emu_g2c_add(const uint8_t* p192, int p_inf, const uint8_t* q192, int q_inf, uint8_t* out192) {
  uint32_t g[G2C_WORDS] = {};
  g2c_st_point(g, emu_lift(p_inf ? g2a{} : load_g2(p192), p_inf, 3));
  g2c_st_q(g, emu_lift(q_inf ? g2a{} : load_g2(q192), q_inf, 5));
  g2c_host_add(g);
  g2a o;
  if (!jac_to_aff(g2c_ld_point(g), o)) return 0;
  g2a_to_be192(o, out192);
  return 1;
}
// the cooperative Miller loop's phase schedule (gt_wave.hpp gtw_miller_schedule: the next step's line on lanes < 64, f
// on lanes 64 .. 191), lanes run in turn within each phase
void emu_gtw_miller(const uint8_t* p96, const uint8_t* q192, uint8_t* out576) {
  static uint32_t F[GTW_FP12], QA[4 * BLS_NL], TB[20 * BLS_NL], L0[GTW_FP12], L1[GTW_FP12], S[108 * BLS_NL],
      S2[28 * BLS_NL];
  const g1a P = load_g1(p96);
  const g2a Q = load_g2(q192);
  lds_st(QA, 0, Q.x.c0);
  lds_st(QA, 1, Q.x.c1);
  lds_st(QA, 2, Q.y.c0);
  lds_st(QA, 3, Q.y.c1);
  gtw_miller_schedule(
      [&](auto&& phase) {
        for (uint32_t t = 0; t < GTW_MILLER_LANES; t++) phase(t);
      },
      F, QA, P.x, P.y, TB, L0, L1, S, S2);
  // w-basis coefficient k -> tower slot (c0.c0, c1.c0, c0.c1, c1.c1, c0.c2, c1.c2)[k]
  fp12 f;
  fp2* slot[6] = {&f.c0.c0, &f.c1.c0, &f.c0.c1, &f.c1.c1, &f.c0.c2, &f.c1.c2};
  for (int k = 0; k < 6; k++) *slot[k] = fp2_make(lds_ld(F, 2 * k), lds_ld(F, 2 * k + 1));
  store12(f, out576);
}
#if defined(BLS_COUNT_OPS)
// bucket MSM over n distinct points (the count covers the MSM only, not the point loads)
void emu_stage_sig_msm(const uint8_t* pts192, int n) {
  static g2a P[4096];
  static uint64_t w[4096];
  uint64_t z = 0x1234567887654321ull;
  for (int i = 0; i < n; i++) {
    P[i] = load_g2(pts192 + 192 * (size_t)i);
    z = z * 6364136223846793005ull + 1442695040888963407ull;
    w[i] = z;
  }
  bls_count_mul = bls_count_sqr = bls_count_half = 0;
  (void)emu_msm_core(P, w, nullptr, n);
}
void emu_count_reset() { bls_count_mul = bls_count_sqr = bls_count_half = 0; }
// lazy-reduction Fp2 products count half-products and reductions (each half a multiplication): reported in mul
unsigned long long emu_count_mul() { return bls_count_mul + bls_count_half / 2; }
unsigned long long emu_count_sqr() { return bls_count_sqr; }
// kernel-shaped stages (same calls as kernels.hip)
void emu_stage_sig_scale(const uint8_t* sig192, uint64_t r) { (void)jac_mul_u64(load_g2(sig192), r); }
void emu_stage_pk_finish(const uint8_t* pk96, uint64_t r) {
  g1a a;
  (void)jac_to_aff(jac_mul_u64(load_g1(pk96), r), a);
}
void emu_stage_sig_scale_w(const uint8_t* sig192, uint64_t w) { (void)emu_mul_scalar_word(jac_from_aff(load_g2(sig192)), w); }
void emu_stage_pk_finish_w(const uint8_t* pk96, uint64_t w) {
  g1a a;
  (void)jac_to_aff(emu_mul_scalar_word(jac_from_aff(load_g1(pk96)), w), a);
}
// Miller stage as the kernels split it: lines per message (k_miller_lines), accumulation per chunk of k
// pairings with shared squarings (k_miller_acc)
void emu_stage_miller_lines(const uint8_t* q192) {
  const g2a Q = load_g2(q192);
  g2proj T;
  T.x = Q.x;
  T.y = Q.y;
  T.z = fp2_one();
  int bit = 62;
  bool add_next = false;
  for (int s = 0; s < MILLER_STEPS; s++) {
    line3 L;
    if (!add_next) {
      miller_dbl_line(T, L);
      add_next = (BLS_Z_ABS >> bit) & 1ull;
      bit--;
    } else {
      miller_add_line(T, Q, L);
      add_next = false;
    }
  }
}
void emu_stage_miller_acc(const uint8_t* pk96, const uint8_t* q192, int k) {
  const g1a P = load_g1(pk96);
  const g2a Q = load_g2(q192);
  line3 L;
  L.l0 = Q.x;
  L.c1 = Q.y;
  L.c4 = Q.x;
  fp12 f = fp12_one();
  int bit = 62;
  bool add_next = false;
  for (int s = 0; s < MILLER_STEPS; s++) {
    if (!add_next && s != 0) f = fp12_sqr(f);
    for (int j = 0; j < k; j++) f = fp12_mul_by_014(f, L.l0, fp2_mul_fp(L.c1, P.x), fp2_mul_fp(L.c4, P.y));
    if (!add_next) {
      add_next = (BLS_Z_ABS >> bit) & 1ull;
      bit--;
    } else {
      add_next = false;
    }
  }
}
void emu_stage_group_sig_miller(const uint8_t* sig192, int n) {
  g2j S = jac_infinity<fp2>();
  g2j s = jac_from_aff(load_g2(sig192));
  g2j t = jac_dbl(s);
  for (int i = 0; i < n; i++) S = jac_add(S, (i & 1) ? s : t);
  g2a Sa;
  jac_to_aff(S, Sa);
  g1a ng;
  ng.x = G1_GEN_X;
  ng.y = G1_NEG_GEN_Y;
  (void)miller_loop(ng, Sa);
}
void emu_stage_group_finish(const uint8_t* f576, int n) {
  fp12 f = load12(f576);
  fp12 acc = f;
  for (int i = 0; i < n; i++) acc = fp12_mul(acc, f);
  (void)final_exponentiation(acc);
}
void emu_stage_pk_aggregate(const uint8_t* pk96, int n) {
  g1a p = load_g1(pk96);
  g1j acc = jac_infinity<fp>();
  g1j two = jac_dbl(jac_from_aff(p));
  g1a p2;
  jac_to_aff(two, p2);
  for (int i = 0; i < n; i++) acc = jac_add_aff(acc, (i & 1) ? p : p2);
}
#endif
// KeyValidate (48- or 96-byte pubkey) -> status, 96-byte uncompressed
int emu_key_validate(const uint8_t* b, uint32_t len, uint8_t* out96) {
  g1a p;
  int st = pk_key_validate(b, len, p);
  if (st == 0) g1a_to_be96(p, out96);
  return st;
}
int emu_g1_in_subgroup(const uint8_t* pk96) { return g1_in_subgroup(load_g1(pk96)) ? 1 : 0; }
void emu_fp_mul(const uint8_t* a, const uint8_t* b, uint8_t* out) { fp_to_be48(fp_mul(load_mont(a), load_mont(b)), out); }
void emu_fp_sqr(const uint8_t* a, uint8_t* out) { fp_to_be48(fp_sqr(load_mont(a)), out); }
void emu_fp_add(const uint8_t* a, const uint8_t* b, uint8_t* out) { fp_to_be48(fp_add(load_mont(a), load_mont(b)), out); }
void emu_fp_sub(const uint8_t* a, const uint8_t* b, uint8_t* out) { fp_to_be48(fp_sub(load_mont(a), load_mont(b)), out); }
void emu_fp_inv(const uint8_t* a, uint8_t* out) { fp_to_be48(fp_inv(load_mont(a)), out); }
void emu_fp_half(const uint8_t* a, uint8_t* out) { fp_to_be48(fp_half(load_mont(a)), out); }
int emu_fp2_sqrt(const uint8_t* a, uint8_t* out) {
  fp2 r;
  bool ok = fp2_sqrt(load2(a), r);
  store2(r, out);
  return ok;
}
void emu_fp2_mul(const uint8_t* a, const uint8_t* b, uint8_t* out) { store2(fp2_mul(load2(a), load2(b)), out); }
void emu_fp2_sqr(const uint8_t* a, uint8_t* out) { store2(fp2_sqr(load2(a)), out); }
void emu_fp2_inv(const uint8_t* a, uint8_t* out) { store2(fp2_inv(load2(a)), out); }
int emu_sig_decode(const uint8_t* b, uint32_t len, uint8_t* out192, int* inf) {
  g2a p;
  bool is_inf;
  int st = sig_decode(b, len, p, is_inf);
  *inf = is_inf;
  if (st == 0 && !is_inf) g2a_to_be192(p, out192);
  return st;
}
int emu_pk_decode(const uint8_t* b, uint8_t* out96) {
  g1a p;
  bool inf;
  int st = pk_decode96(b, p, inf);
  if (st == 0 && !inf) g1a_to_be96(p, out96);
  return st;
}
void emu_expand_message(const uint8_t* msg, uint8_t* out256) {
  uint32_t w[64];
  expand_message_xmd_32(msg, w);
  for (int i = 0; i < 64; i++)
    for (int j = 0; j < 4; j++) out256[4 * i + j] = (uint8_t)(w[i] >> (24 - 8 * j));
}
void emu_hash_to_field(const uint8_t* msg, uint8_t* out192) {
  fp2 u0, u1;
  hash_to_field_fp2x2(msg, u0, u1);
  store2(u0, out192);
  store2(u1, out192 + 96);
}
int emu_hash_to_g2(const uint8_t* msg, uint8_t* out192) {
  g2j h = hash_to_g2_jac(msg);
  g2a a;
  if (!jac_to_aff(h, a)) return 0;
  g2a_to_be192(a, out192);
  return 1;
}
int emu_g2_in_subgroup(const uint8_t* p192) { return g2_in_subgroup(load_g2(p192)); }
// the kernel's form (k_sig.hip): P re-read from memory along the chain
int emu_g2_in_subgroup_ld(const uint8_t* p192) {
  const g2a p = load_g2(p192);
  return g2_in_subgroup_ld([&] { return p; });
}
int emu_g2_mul_u64(const uint8_t* p192, uint64_t k, uint8_t* out192) {
  g2a a;
  if (!jac_to_aff(jac_mul_u64(load_g2(p192), k), a)) return 0;
  g2a_to_be192(a, out192);
  return 1;
}
int emu_g1_mul_u64(const uint8_t* p96, uint64_t k, uint8_t* out96) {
  g1a a;
  if (!jac_to_aff(jac_mul_u64(load_g1(p96), k), a)) return 0;
  g1a_to_be96(a, out96);
  return 1;
}
void emu_miller(const uint8_t* p96, const uint8_t* q192, uint8_t* out576) { store12(miller_loop(load_g1(p96), load_g2(q192)), out576); }
// two-pass form of the pipeline kernels (k_miller_lines + k_miller_acc)
void emu_miller2(const uint8_t* p96, const uint8_t* q192, uint8_t* out576) {
  const g1a P = load_g1(p96);
  const g2a Q = load_g2(q192);
  static line3 L[MILLER_STEPS];
  g2proj T;
  T.x = Q.x;
  T.y = Q.y;
  T.z = fp2_one();
  for (int s = 0; s < MILLER_STEPS; s++) {
    if (miller_step_is_add(s)) miller_add_line(T, Q, L[s]);
    else miller_dbl_line(T, L[s]);
  }
  fp12 f = fp12_one();
  for (int s = 0; s < MILLER_STEPS; s++) f = miller_acc_step(f, s, miller_step_is_add(s), L[s], P.x, P.y);
  store12(fp12_conj(f), out576);
}
void emu_final_exp(const uint8_t* f576, uint8_t* out576) { store12(final_exponentiation(load12(f576)), out576); }
void emu_fp12_mul(const uint8_t* a, const uint8_t* b, uint8_t* out) { store12(fp12_mul(load12(a), load12(b)), out); }
void emu_fp12_sqr(const uint8_t* a, uint8_t* out) { store12(fp12_sqr(load12(a)), out); }
void emu_fp12_inv(const uint8_t* a, uint8_t* out) { store12(fp12_inv(load12(a)), out); }
void emu_fp12_cyc_sqr(const uint8_t* a, uint8_t* out) { store12(fp12_cyclotomic_sqr(load12(a)), out); }
void emu_fp12_frob1(const uint8_t* a, uint8_t* out) { store12(fp12_frob1(load12(a)), out); }
}
extern "C" void emu_fp2_mul_lazy(const uint8_t* a, const uint8_t* b, uint8_t* out) {
  const fp2 x = load2(a), y = load2(b);
  store2(fp2_mul_lazy_body(x.c0, x.c1, y.c0, y.c1), out);
}
// raw-limb entry: a0, a1, b0, b1 as 14 uint32 limbs each (any limb pattern the bounds allow), out 28 limbs
extern "C" void emu_fp2_mul_lazy_limbs(const uint32_t* in56, uint32_t* out28) {
  fp a0, a1, b0, b1;
  for (int i = 0; i < BLS_NL; i++) {
    a0.l[i] = in56[i];
    a1.l[i] = in56[14 + i];
    b0.l[i] = in56[28 + i];
    b1.l[i] = in56[42 + i];
  }
  const fp2 r = fp2_mul_lazy_body(a0, a1, b0, b1);
  for (int i = 0; i < BLS_NL; i++) {
    out28[i] = r.c0.l[i];
    out28[14 + i] = r.c1.l[i];
  }
}
// hash_to_G2 as the pipeline runs it: the two maps on separate lanes (hash_to_g2_map_j), then sum + cofactor
// clearing (k_hash.hip k_hash_map / k_hash_clear)
extern "C" int emu_hash_to_g2_split(const uint8_t* msg, uint8_t* out192) {
  h2c_prep h;
  hash_to_g2_prep(msg, h);
  const fp2 dinv = fp2_inv(h.d);
  g2j slot[2];  // as k_hash_clear: slots 0 and 1 share one place (the LDS base point), slot 2 its own
  slot[0] = jac_add(hash_to_g2_map_j(h, dinv, 0), hash_to_g2_map_j(h, dinv, 1));
  const g2j H = clear_cofactor_g2_slots([&](int k) { return slot[k == 2 ? 1 : 0]; },
                                        [&](int k, const g2j& v) { slot[k == 2 ? 1 : 0] = v; });
  g2a a;
  if (!jac_to_aff(H, a)) return 0;
  g2a_to_be192(a, out192);
  return 1;
}

// fp_lc at the edges of its contract (raw 14-limb terms, normalized, values <= 2p): 7 positive and 8 negative unit
// terms, and weighted terms 2, -3, 5, -4, 1
extern "C" void emu_fp_lc_7p8n(const uint32_t* in, uint32_t* out14) {
  fp x[15];
  for (int k = 0; k < 15; k++)
    for (int i = 0; i < BLS_NL; i++) x[k].l[i] = in[14 * k + i];
  const fp r = fp_lc(T<1>(x[0]), T<1>(x[1]), T<1>(x[2]), T<1>(x[3]), T<1>(x[4]), T<1>(x[5]), T<1>(x[6]), T<-1>(x[7]),
                     T<-1>(x[8]), T<-1>(x[9]), T<-1>(x[10]), T<-1>(x[11]), T<-1>(x[12]), T<-1>(x[13]), T<-1>(x[14]));
  for (int i = 0; i < BLS_NL; i++) out14[i] = r.l[i];
}
extern "C" void emu_fp_lc_weighted(const uint32_t* in, uint32_t* out14) {
  fp x[5];
  for (int k = 0; k < 5; k++)
    for (int i = 0; i < BLS_NL; i++) x[k].l[i] = in[14 * k + i];
  const fp r = fp_lc(T<2>(x[0]), T<-3>(x[1]), T<5>(x[2]), T<-4>(x[3]), T<1>(x[4]));
  for (int i = 0; i < BLS_NL; i++) out14[i] = r.l[i];
}

// k_pk_aggregate's schedule on the host: 64 strided lane sums of mixed additions, then the pairwise jac_add tree
extern "C" int emu_g1_aggregate(const uint8_t* pks96, int n, uint8_t* out96) {
  g1j acc[64];
  for (int l = 0; l < 64; l++) acc[l] = jac_infinity<fp>();
  for (int k = 0; k < n; k++) acc[k % 64] = jac_add_aff(acc[k % 64], load_g1(pks96 + 96 * k));
  for (int s = 32; s >= 1; s >>= 1)
    for (int l = 0; l < s; l++) acc[l] = jac_add(acc[l], acc[l + s]);
  g1a r;
  if (!jac_to_aff(acc[0], r)) return 0;
  fp_to_be48(r.x, out96);
  fp_to_be48(r.y, out96 + 48);
  return 1;
}

// fp2_sqr at the edge of its operand contract: raw normalized limbs, values <= 4p (fp2_add_norm of two stored values);
// the old fp_sub form underflowed for a1 - a0 > 2p
extern "C" void emu_fp2_sqr_limbs(const uint32_t* in28, uint32_t* out28) {
  fp2 a;
  for (int i = 0; i < BLS_NL; i++) {
    a.c0.l[i] = in28[i];
    a.c1.l[i] = in28[14 + i];
  }
  const fp2 r = fp2_sqr(a);
  for (int i = 0; i < BLS_NL; i++) {
    out28[i] = r.c0.l[i];
    out28[14 + i] = r.c1.l[i];
  }
}

// f * l_a * l_b two ways: two sparse products (fp12_mul_by_014) and the line-pair form (line_pair, then
// fp12_mul_by_line2); 1 when they are equal mod p.  in: f (576 B), then the six Fp2 line coefficients (6 x 96 B).
extern "C" int emu_line_pair_check(const uint8_t* f576, const uint8_t* lines576) {
  const fp12 f = load12(f576);
  const fp2 a0 = load2(lines576), a1 = load2(lines576 + 96), a4 = load2(lines576 + 192);
  const fp2 b0 = load2(lines576 + 288), b1 = load2(lines576 + 384), b4 = load2(lines576 + 480);
  const fp12 x = fp12_mul_by_014(fp12_mul_by_014(f, a0, a1, a4), b0, b1, b4);
  const fp12 y = fp12_mul_by_line2(f, line_pair(a0, a1, a4, b0, b1, b4));
  uint8_t bx[576], by[576];
  store12(x, bx);
  store12(y, by);
  for (int i = 0; i < 576; i++)
    if (bx[i] != by[i]) return 0;
  return 1;
}
// the schoolbook-offset Fp2 product body on raw limbs (same layout as emu_fp2_mul_lazy_limbs)
extern "C" void emu_fp2_mul_sb_limbs(const uint32_t* in56, uint32_t* out28) {
  fp a0, a1, b0, b1;
  for (int i = 0; i < BLS_NL; i++) {
    a0.l[i] = in56[i];
    a1.l[i] = in56[14 + i];
    b0.l[i] = in56[28 + i];
    b1.l[i] = in56[42 + i];
  }
  const fp2 r = fp2_mul_sb_body(a0, a1, b0, b1);
  for (int i = 0; i < BLS_NL; i++) {
    out28[i] = r.c0.l[i];
    out28[14 + i] = r.c1.l[i];
  }
}
