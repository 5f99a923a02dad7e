// Element-wise test hooks behind blsgpu_debug_op (stage parity tests and workload generation).
#include "k_common.hpp"
#include "gt_wave.hpp"

__device__ fp dbg_load_fp(const uint8_t* b) {
  fp x;
  fp_from_be48_plain(b, x, 0xff);
  return fp_to_mont(x);
}
__device__ fp2 dbg_load_fp2(const uint8_t* b) { return fp2_make(dbg_load_fp(b + 48), dbg_load_fp(b)); }
__device__ g2a dbg_load_g2(const uint8_t* b) {
  g2a p;
  p.x = dbg_load_fp2(b);
  p.y = dbg_load_fp2(b + 96);
  return p;
}
__device__ g1a dbg_load_g1(const uint8_t* b) {
  g1a p;
  p.x = dbg_load_fp(b);
  p.y = dbg_load_fp(b + 48);
  return p;
}
__device__ void dbg_store_fp12(const fp12& f, uint8_t* b) {
  const fp2* c[6] = {&f.c0.c0, &f.c0.c1, &f.c0.c2, &f.c1.c0, &f.c1.c1, &f.c1.c2};
  for (int k = 0; k < 6; k++) {
    fp_to_be48(c[k]->c0, b + 96 * k);
    fp_to_be48(c[k]->c1, b + 96 * k + 48);
  }
}
__device__ fp12 dbg_load_fp12(const uint8_t* b) {
  fp12 f;
  fp2* c[6] = {&f.c0.c0, &f.c0.c1, &f.c0.c2, &f.c1.c0, &f.c1.c1, &f.c1.c2};
  for (int k = 0; k < 6; k++) {
    c[k]->c0 = dbg_load_fp(b + 96 * k);
    c[k]->c1 = dbg_load_fp(b + 96 * k + 48);
  }
  return f;
}

__global__ __launch_bounds__(WAVE) void k_debug_op(int op, uint32_t n, const uint8_t* in, uint32_t in_stride,
                                                   uint8_t* out, uint32_t out_stride, int32_t* status) {
  uint32_t i = blockIdx.x * WAVE + threadIdx.x;
  if (i >= n) return;
  const uint8_t* a = in + (size_t)i * in_stride;
  uint8_t* o = out + (size_t)i * out_stride;
  int st = 0;
  switch (op) {
    case 0:
      fp_to_be48(fp_mul(dbg_load_fp(a), dbg_load_fp(a + 48)), o);
      break;
    case 1: {
      uint32_t len = (uint32_t)a[192] | ((uint32_t)a[193] << 8);
      g2a p;
      bool inf;
      st = sig_decode(a, len, p, inf);
      if (st == 0 && !inf) g2a_to_be192(p, o);
      if (st == 0 && inf) st = -1;
      break;
    }
    case 2: {
      g2a p;
      st = jac_to_aff(hash_to_g2_jac(a), p) ? 0 : -1;
      if (st == 0) g2a_to_be192(p, o);
      break;
    }
    case 3:
      dbg_store_fp12(miller_loop(dbg_load_g1(a), dbg_load_g2(a + 96)), o);
      break;
    case 4:
      dbg_store_fp12(final_exponentiation(dbg_load_fp12(a)), o);
      break;
    case 5: {
      uint64_t k = 0;
      for (int j = 0; j < 8; j++) k |= (uint64_t)a[96 + j] << (8 * j);
      g1a r;
      st = jac_to_aff(jac_mul_u64(dbg_load_g1(a), k), r) ? 0 : -1;
      if (st == 0) g1a_to_be96(r, o);
      break;
    }
    case 6: {
      uint64_t k = 0;
      for (int j = 0; j < 8; j++) k |= (uint64_t)a[192 + j] << (8 * j);
      g2a r;
      st = jac_to_aff(jac_mul_u64(dbg_load_g2(a), k), r) ? 0 : -1;
      if (st == 0) g2a_to_be192(r, o);
      break;
    }
    case 7: {  // sign: sk (32 B big-endian) || msg (32 B) -> compressed signature (96 B)
      uint32_t w[8];
      for (int j = 0; j < 8; j++)
        w[j] = ((uint32_t)a[31 - 4 * j]) | ((uint32_t)a[30 - 4 * j] << 8) | ((uint32_t)a[29 - 4 * j] << 16) |
               ((uint32_t)a[28 - 4 * j] << 24);
      g2j h = hash_to_g2_jac(a + 32);
      g2a ha;
      st = jac_to_aff(h, ha) ? 0 : -1;
      g2a s;
      if (st == 0) st = jac_to_aff(jac_mul_words(jac_from_aff(ha), w, 8), s) ? 0 : -1;
      if (st == 0) g2a_compress(s, o);
      break;
    }
    case 8: {  // sk_to_pk: sk (32 B big-endian) -> uncompressed pubkey (96 B)
      uint32_t w[8];
      for (int j = 0; j < 8; j++)
        w[j] = ((uint32_t)a[31 - 4 * j]) | ((uint32_t)a[30 - 4 * j] << 8) | ((uint32_t)a[29 - 4 * j] << 16) |
               ((uint32_t)a[28 - 4 * j] << 24);
      g1a g;
      g.x = G1_GEN_X;
      g.y = G1_GEN_Y;
      g1a pk;
      st = jac_to_aff(jac_mul_words(jac_from_aff(g), w, 8), pk) ? 0 : -1;
      if (st == 0) g1a_to_be96(pk, o);
      break;
    }
    case 9: {  // batch-scalar-word multiple of a G2 point: 192 B || word (8 B LE) -> 192 B (table after it)
      uint64_t w = 0;
      for (int j = 0; j < 8; j++) w |= (uint64_t)a[192 + j] << (8 * j);
      g2a r;
      uint32_t* tab = reinterpret_cast<uint32_t*>(o + 192);
      st = jac_to_aff(jac_mul_scalar_word(jac_from_aff(dbg_load_g2(a)), w, tab, 1, 0), r) ? 0 : -1;
      if (st == 0) g2a_to_be192(r, o);
      break;
    }
    case 10: {  // the same in G1: 96 B || word -> 96 B (table after it)
      uint64_t w = 0;
      for (int j = 0; j < 8; j++) w |= (uint64_t)a[96 + j] << (8 * j);
      g1a r;
      uint32_t* tab = reinterpret_cast<uint32_t*>(o + 96);
      st = jac_to_aff(jac_mul_scalar_word(jac_from_aff(dbg_load_g1(a)), w, tab, 1, 0), r) ? 0 : -1;
      if (st == 0) g1a_to_be96(r, o);
      break;
    }
    case 11: {  // fp_lc of raw limbs (15 x 14 LE words): 7 positive, 8 negative unit terms -> 14 words
      const uint32_t* w = reinterpret_cast<const uint32_t*>(a);
      fp x[15];
      for (int k = 0; k < 15; k++)
        for (int j = 0; j < BLS_NL; j++) x[k].l[j] = w[14 * k + j];
      const fp r = fp_lc(T<1>(x[0]), T<1>(x[1]), T<1>(x[2]), T<1>(x[3]), T<1>(x[4]), T<1>(x[5]), T<1>(x[6]),
                         T<-1>(x[7]), T<-1>(x[8]), T<-1>(x[9]), T<-1>(x[10]), T<-1>(x[11]), T<-1>(x[12]), T<-1>(x[13]),
                         T<-1>(x[14]));
      uint32_t* ow = reinterpret_cast<uint32_t*>(o);
      for (int j = 0; j < BLS_NL; j++) ow[j] = r.l[j];
      break;
    }
    default:
      st = -2;
  }
  status[i] = st;
}

// Workgroup-cooperative GT engine (gt_wave.hpp), one element per 128-lane block:
//   op 16: final exponentiation of an Fp12 (576 B) -> Fp12
//   op 17: Miller loop of (P: G1 affine 96 B, Q: G2 affine 192 B) -> Fp12
__global__ __launch_bounds__(GTW_MILLER_LANES) void k_debug_gt(int op, const uint8_t* in, uint32_t in_stride, uint8_t* out,
                                                         uint32_t out_stride, int32_t* status) {
  __shared__ GtwLds sh;
  const uint32_t i = blockIdx.x, t = threadIdx.x;
  const uint8_t* a = in + (size_t)i * in_stride;
  uint8_t* o = out + (size_t)i * out_stride;
  if (op == 16) {
    if (t == 0) gtw_from_reg(sh.F, dbg_load_fp12(a));
    gtw_sync();
    gtw_final_exp(sh.F, sh.W, sh.S, t);
  } else {
    if (t == 0) {
      const g1a P = dbg_load_g1(a);
      const g2a Q = dbg_load_g2(a + 96);
      lds_st(sh.QA, 0, Q.x.c0);
      lds_st(sh.QA, 1, Q.x.c1);
      lds_st(sh.QA, 2, Q.y.c0);
      lds_st(sh.QA, 3, Q.y.c1);
      lds_st(sh.L, 0, P.x);
      lds_st(sh.L, 1, P.y);
    }
    gtw_sync();
    const fp xP = lds_ld(sh.L, 0), yP = lds_ld(sh.L, 1);
    gtw_sync();
    gtw_miller_loop(sh.F, sh.QA, xP, yP, sh.TB, sh.L, sh.L1, sh.S, sh.S2, t);
  }
  if (t == 0) {
    dbg_store_fp12(gtw_to_reg(sh.F), o);
    status[i] = 0;
  }
}

// Lane-pair G2 arithmetic against the one-lane forms (op 18; fp2x.hpp), lane pair per element: input P, Q affine
// (192 B each).  The pair builds P, Q in Jacobian form with Z != 1 (P scaled by l = 2 + i, Q by l + 1), computes
// P + Q, P + P (the addition's doubling branch), P + (-P) (its infinity branch), P + O, O + Q, 2P, P + Q_affine,
// psi(P), psi^2(P), [|z|]P and the Fp2 product / square of P.x, Q.y; lane 0 gathers each result and compares it with
// the same operation on one lane (jac_eq, or Fp2 equality).  status = bit k set when case k differs; out = [|z|]P
// affine (192 B) from the pair's result, for an oracle check.
__global__ __launch_bounds__(WAVE) void k_debug_pairs(uint32_t n, const uint8_t* in, uint32_t in_stride, uint8_t* out,
                                                      uint32_t out_stride, int32_t* status) {
  const uint32_t q = blockIdx.x * WAVE + threadIdx.x, i = q >> 1, k = q & 1;
  if (i >= n) return;
  const uint8_t* a = in + (size_t)i * in_stride;
  const g2a Pa = dbg_load_g2(a), Qa = dbg_load_g2(a + 192);
  fp l1 = fp_zero();
  l1.l[0] = 2 + i;
  l1 = fp_to_mont(l1);
  const fp2 lp = fp2_make(l1, FP_ONE), lq = fp2_make(fp_add(l1, FP_ONE), FP_ONE);
  auto scale = [](const g2a& p, const fp2& l) {
    g2j r;
    const fp2 l2 = fp2_sqr(l);
    r.x = fp2_mul(p.x, l2);
    r.y = fp2_mul(p.y, fp2_mul(l2, l));
    r.z = l;
    return r;
  };
  const g2j P = scale(Pa, lp), Q = scale(Qa, lq), O = jac_infinity<fp2>();
  auto x_of = [&](const g2j& v) {
    g2jx r;
    r.x = fp2x_of(v.x);
    r.y = fp2x_of(v.y);
    r.z = fp2x_of(v.z);
    return r;
  };
  auto gather = [&](const g2jx& v) {  // both lanes: the full point
    g2j r;
    const fp ox = fp_swap(v.x.v), oy = fp_swap(v.y.v), oz = fp_swap(v.z.v);
    r.x = k ? fp2_make(ox, v.x.v) : fp2_make(v.x.v, ox);
    r.y = k ? fp2_make(oy, v.y.v) : fp2_make(v.y.v, oy);
    r.z = k ? fp2_make(oz, v.z.v) : fp2_make(v.z.v, oz);
    return r;
  };
  auto gather2 = [&](const fp2x& v) {
    const fp o2 = fp_swap(v.v);
    return k ? fp2_make(o2, v.v) : fp2_make(v.v, o2);
  };
  const g2jx Px = x_of(P), Qx = x_of(Q), Ox = x_of(O);
  aff<fp2x> Qax;
  Qax.x = fp2x_of(Qa.x);
  Qax.y = fp2x_of(Qa.y);
  const g2j r0 = gather(jac_add(Px, Qx)), r1 = gather(jac_add(Px, Px)), r2 = gather(jac_add(Px, jac_neg(Px))),
            r3 = gather(jac_add(Px, Ox)), r4 = gather(jac_add(Ox, Qx)), r5 = gather(jac_dbl(Px)),
            r6 = gather(jac_add_aff(Px, Qax)), r7 = gather(g2_psi(Px)), r8 = gather(g2_psi2(Px)),
            r9 = gather(jac_mul_zabs(Px));
  const fp2 m0 = gather2(F_mul(Px.x, Qx.y)), m1 = gather2(F_sqr(Px.x));
  if (k == 0) {
    int st = 0;
    st |= jac_eq(r0, jac_add(P, Q)) ? 0 : 1;
    st |= jac_eq(r1, jac_dbl(P)) ? 0 : 2;
    st |= jac_is_inf(r2) ? 0 : 4;
    st |= jac_eq(r3, P) ? 0 : 8;
    st |= jac_eq(r4, Q) ? 0 : 16;
    st |= jac_eq(r5, jac_dbl(P)) ? 0 : 32;
    st |= jac_eq(r6, jac_add_aff(P, Qa)) ? 0 : 64;
    st |= jac_eq(r7, g2_psi(P)) ? 0 : 128;
    st |= jac_eq(r8, g2_psi2(P)) ? 0 : 256;
    st |= jac_eq(r9, jac_mul_zabs(P)) ? 0 : 512;
    st |= fp2_eq(m0, fp2_mul(P.x, Q.y)) ? 0 : 1024;
    st |= fp2_eq(m1, fp2_sqr(P.x)) ? 0 : 2048;
    g2a z;
    if (jac_to_aff(r9, z)) g2a_to_be192(z, out + (size_t)i * out_stride);
    status[i] = st;
  }
}

static inline dim3 grid_for(uint32_t n) { return dim3((n + WAVE - 1) / WAVE); }

void launch_debug_op(int op, uint32_t n, const uint8_t* in, uint32_t in_stride, uint8_t* out, uint32_t out_stride,
                     int32_t* status, hipStream_t s) {
  if (!n) return;
  if (op == 16 || op == 17)
    hipLaunchKernelGGL(k_debug_gt, dim3(n), dim3(GTW_MILLER_LANES), 0, s, op, in, in_stride, out, out_stride, status);
  else if (op == 18)
    hipLaunchKernelGGL(k_debug_pairs, grid_for(2 * n), dim3(WAVE), 0, s, n, in, in_stride, out, out_stride, status);
  else
    hipLaunchKernelGGL(k_debug_op, grid_for(n), dim3(WAVE), 0, s, op, n, in, in_stride, out, out_stride, status);
}
