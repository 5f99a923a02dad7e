// HIP kernels of the BLS12-381 signature-set verification pipeline for MI355X (gfx950).
//
// One lane per signature set (or per batch group), SoA limb-major intermediates in HBM so that the 64
// lanes of a wave touch 64 consecutive words per limb (fully coalesced):
//   k_sig_decode     A8   Signature.fromBytes(.., validate=true): decompress + psi subgroup check
//   k_hash_to_g2     A11  hash_to_G2 (expand_message_xmd / SSWU / iso3 / clear_cofactor)
//   k_pk_aggregate   A4   PublicKey.aggregate over the device pubkey table (one wave per set)
//   k_pk_finish      A9   r_i * pk_i (64-bit random scalar), to affine
//   k_sig_scale      A9   r_i * sig_i
//   k_miller_sets    A12  f_i = MillerLoop(r_i pk_i, H(m_i))
//   k_group_sig_miller   per batch group: S = sum r_i sig_i, f_g = MillerLoop(-g1, S)
//   k_group_finish       per batch group: FinalExp(f_g * prod f_i) == 1
// (A-numbers: SURVEY.md section 8a rows.)
#include "kernels.h"
#include "ops.hpp"

#define WAVE 64

__device__ __forceinline__ fp ld_fp(const uint32_t* p, uint32_t n, uint32_t i, int w0) {
  fp r;
#pragma unroll
  for (int l = 0; l < BLS_NL; l++) r.l[l] = p[(size_t)(w0 + l) * n + i];
  return r;
}
__device__ __forceinline__ void st_fp(uint32_t* p, uint32_t n, uint32_t i, int w0, const fp& v) {
#pragma unroll
  for (int l = 0; l < BLS_NL; l++) p[(size_t)(w0 + l) * n + i] = v.l[l];
}
__device__ __forceinline__ fp2 ld_fp2(const uint32_t* p, uint32_t n, uint32_t i, int w0) {
  return fp2_make(ld_fp(p, n, i, w0), ld_fp(p, n, i, w0 + W_FP));
}
__device__ __forceinline__ void st_fp2(uint32_t* p, uint32_t n, uint32_t i, int w0, const fp2& v) {
  st_fp(p, n, i, w0, v.c0);
  st_fp(p, n, i, w0 + W_FP, v.c1);
}
__device__ __forceinline__ g2a ld_g2a(const uint32_t* p, uint32_t n, uint32_t i) {
  g2a r;
  r.x = ld_fp2(p, n, i, 0);
  r.y = ld_fp2(p, n, i, 2 * W_FP);
  return r;
}
__device__ __forceinline__ void st_g2a(uint32_t* p, uint32_t n, uint32_t i, const g2a& v) {
  st_fp2(p, n, i, 0, v.x);
  st_fp2(p, n, i, 2 * W_FP, v.y);
}
__device__ __forceinline__ g2j ld_g2j(const uint32_t* p, uint32_t n, uint32_t i) {
  g2j r;
  r.x = ld_fp2(p, n, i, 0);
  r.y = ld_fp2(p, n, i, 2 * W_FP);
  r.z = ld_fp2(p, n, i, 4 * W_FP);
  return r;
}
__device__ __forceinline__ void st_g2j(uint32_t* p, uint32_t n, uint32_t i, const g2j& v) {
  st_fp2(p, n, i, 0, v.x);
  st_fp2(p, n, i, 2 * W_FP, v.y);
  st_fp2(p, n, i, 4 * W_FP, v.z);
}
__device__ __forceinline__ g1a ld_g1a(const uint32_t* p, uint32_t n, uint32_t i) {
  g1a r;
  r.x = ld_fp(p, n, i, 0);
  r.y = ld_fp(p, n, i, W_FP);
  return r;
}
__device__ __forceinline__ void st_g1a(uint32_t* p, uint32_t n, uint32_t i, const g1a& v) {
  st_fp(p, n, i, 0, v.x);
  st_fp(p, n, i, W_FP, v.y);
}
__device__ __forceinline__ g1j ld_g1j(const uint32_t* p, uint32_t n, uint32_t i) {
  g1j r;
  r.x = ld_fp(p, n, i, 0);
  r.y = ld_fp(p, n, i, W_FP);
  r.z = ld_fp(p, n, i, 2 * W_FP);
  return r;
}
__device__ __forceinline__ void st_g1j(uint32_t* p, uint32_t n, uint32_t i, const g1j& v) {
  st_fp(p, n, i, 0, v.x);
  st_fp(p, n, i, W_FP, v.y);
  st_fp(p, n, i, 2 * W_FP, v.z);
}
__device__ __forceinline__ fp12 ld_fp12(const uint32_t* p, uint32_t n, uint32_t i) {
  fp12 f;
  f.c0.c0 = ld_fp2(p, n, i, 0);
  f.c0.c1 = ld_fp2(p, n, i, 2 * W_FP);
  f.c0.c2 = ld_fp2(p, n, i, 4 * W_FP);
  f.c1.c0 = ld_fp2(p, n, i, 6 * W_FP);
  f.c1.c1 = ld_fp2(p, n, i, 8 * W_FP);
  f.c1.c2 = ld_fp2(p, n, i, 10 * W_FP);
  return f;
}
__device__ __forceinline__ void st_fp12(uint32_t* p, uint32_t n, uint32_t i, const fp12& f) {
  st_fp2(p, n, i, 0, f.c0.c0);
  st_fp2(p, n, i, 2 * W_FP, f.c0.c1);
  st_fp2(p, n, i, 4 * W_FP, f.c0.c2);
  st_fp2(p, n, i, 6 * W_FP, f.c1.c0);
  st_fp2(p, n, i, 8 * W_FP, f.c1.c1);
  st_fp2(p, n, i, 10 * W_FP, f.c1.c2);
}
__device__ __forceinline__ g1a ld_pktab(const uint32_t* tab, uint32_t idx) {
  const uint4* q = reinterpret_cast<const uint4*>(tab + (size_t)idx * W_PKTAB);
  uint32_t w[W_PKTAB];
#pragma unroll
  for (int k = 0; k < W_PKTAB / 4; k++) {
    uint4 v = q[k];
    w[4 * k] = v.x;
    w[4 * k + 1] = v.y;
    w[4 * k + 2] = v.z;
    w[4 * k + 3] = v.w;
  }
  g1a r;
#pragma unroll
  for (int l = 0; l < BLS_NL; l++) {
    r.x.l[l] = w[l];
    r.y.l[l] = w[BLS_NL + l];
  }
  return r;
}

// [k]P for Jacobian P
template <class F>
__device__ jac<F> jac_mul_u64_j(const jac<F>& P, uint64_t k) {
  jac<F> r = jac_infinity<F>();
  if (k == 0) return r;
  int top = 63;
  while (((k >> top) & 1ull) == 0) top--;
  r = P;
  for (int i = top - 1; i >= 0; i--) {
    r = jac_dbl(r);
    if ((k >> i) & 1ull) r = jac_add(r, P);
  }
  return r;
}

// [k]P for a multi-word scalar (little-endian 32-bit words), used by the workload-generation ops
template <class F>
__device__ jac<F> jac_mul_words(const jac<F>& P, const uint32_t* k, int nw) {
  jac<F> r = jac_infinity<F>();
  for (int i = 32 * nw - 1; i >= 0; i--) {
    r = jac_dbl(r);
    if ((k[i >> 5] >> (i & 31)) & 1u) r = jac_add(r, P);
  }
  return r;
}

// ------------------------------------------------------------------------------------------ kernels
__global__ __launch_bounds__(WAVE) void k_sig_decode(PipelineBuffers b, uint32_t n_sets) {
  uint32_t i = blockIdx.x * WAVE + threadIdx.x;
  if (i >= n_sets) return;
  uint8_t raw[192];
  uint32_t len = b.sig_len[i];
  const uint8_t* src = b.sigs + (size_t)i * b.sig_stride;
  uint32_t cl = len == 96 || len == 192 ? len : 0;
  for (uint32_t k = 0; k < cl; k++) raw[k] = src[k];
  g2a p;
  bool inf = false;
  int st = sig_decode(raw, len, p, inf);
  if (st != BLS_OK || inf) {
    p.x = fp2_zero();
    p.y = fp2_zero();
  }
  st_g2a(b.sig_aff, b.n, i, p);
  b.flags[i] = inf ? SF_SIG_INF : 0;  // sig flags: flags[0, n)
  b.status[i] = (int8_t)st;
}

__global__ __launch_bounds__(WAVE) void k_hash_to_g2(PipelineBuffers b, uint32_t n_sets) {
  uint32_t i = blockIdx.x * WAVE + threadIdx.x;
  if (i >= n_sets) return;
  uint8_t msg[32];
  const uint4* src = reinterpret_cast<const uint4*>(b.msgs + (size_t)i * 32);
  uint4 m0 = src[0], m1 = src[1];
  uint32_t w[8] = {m0.x, m0.y, m0.z, m0.w, m1.x, m1.y, m1.z, m1.w};
#pragma unroll
  for (int k = 0; k < 32; k++) msg[k] = (uint8_t)(w[k >> 2] >> (8 * (k & 3)));
  g2j h = hash_to_g2_jac(msg);
  g2a a;
  bool ok = jac_to_aff(h, a);
  if (!ok) {
    a.x = fp2_zero();
    a.y = fp2_zero();
  }
  st_g2a(b.h_aff, b.n, i, a);
  b.flags[b.n + i] = ok ? 0 : SF_H_INF;  // hash flags: flags[n, 2n)
}

// One wave per set: strided partial sums of table pubkeys, then an LDS tree reduction.
__global__ __launch_bounds__(WAVE) void k_pk_aggregate(PipelineBuffers b, uint32_t n_sets) {
  __shared__ uint32_t red[WAVE * W_G1J];
  uint32_t set = blockIdx.x;
  uint32_t lane = threadIdx.x;
  if (set >= n_sets) return;
  uint32_t first = b.set_pk_first[set], last = b.set_pk_first[set + 1];
  g1j acc = jac_infinity<fp>();
  for (uint32_t k = first + lane; k < last; k += WAVE) {
    uint32_t idx = b.pk_index[k];
    if (idx < b.pk_table_n) acc = jac_add_aff(acc, ld_pktab(b.pk_table, idx));
  }
  uint32_t cnt = last - first;
  if (cnt <= 1) {  // nothing to reduce
    if (lane == 0) st_g1j(b.pk_jac, b.n, set, acc);
    return;
  }
#pragma unroll 1
  for (int s = WAVE / 2; s >= 1; s >>= 1) {
    if (lane >= (uint32_t)s && lane < (uint32_t)(2 * s)) {
#pragma unroll
      for (int l = 0; l < BLS_NL; l++) {
        red[(lane - s) * W_G1J + l] = acc.x.l[l];
        red[(lane - s) * W_G1J + W_FP + l] = acc.y.l[l];
        red[(lane - s) * W_G1J + 2 * W_FP + l] = acc.z.l[l];
      }
    }
    __syncthreads();
    if (lane < (uint32_t)s) {
      g1j o;
#pragma unroll
      for (int l = 0; l < BLS_NL; l++) {
        o.x.l[l] = red[lane * W_G1J + l];
        o.y.l[l] = red[lane * W_G1J + W_FP + l];
        o.z.l[l] = red[lane * W_G1J + 2 * W_FP + l];
      }
      acc = jac_add(acc, o);
    }
    __syncthreads();
  }
  if (lane == 0) st_g1j(b.pk_jac, b.n, set, acc);
}

// r_i * pk_i -> affine.  Bytes mode decodes the 96-byte pubkey; table mode reads k_pk_aggregate's sum.
// pk statuses go to their own array (status[n, 2n)); the host gives them precedence over signature
// statuses because the reference deserializes pubkeys first (worker.ts:39).
__global__ __launch_bounds__(WAVE) void k_pk_finish(PipelineBuffers b, uint32_t n_sets, int8_t* pk_status) {
  uint32_t i = blockIdx.x * WAVE + threadIdx.x;
  if (i >= n_sets) return;
  int st = BLS_OK;
  g1j P;
  if (b.pk_bytes) {
    uint8_t raw[96];
    const uint4* src = reinterpret_cast<const uint4*>(b.pk_bytes + (size_t)i * 96);
#pragma unroll
    for (int k = 0; k < 6; k++) {
      uint4 v = src[k];
      uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int j = 0; j < 16; j++) raw[16 * k + j] = (uint8_t)(w[j >> 2] >> (8 * (j & 3)));
    }
    g1a a;
    bool inf = false;
    st = pk_decode96(raw, a, inf);
    if (st == BLS_OK && inf) st = BLS_PK_IS_INFINITY;
    if (st == BLS_OK) P = jac_from_aff(a);
  } else {
    uint32_t cnt = b.set_pk_first[i + 1] - b.set_pk_first[i];
    if (cnt == 0) {
      st = BLS_EMPTY_AGGREGATE;
    } else {
      P = ld_g1j(b.pk_jac, b.n, i);
      if (jac_is_inf(P)) st = BLS_PK_IS_INFINITY;
    }
  }
  g1a out;
  out.x = fp_zero();
  out.y = fp_zero();
  if (st == BLS_OK) {
    uint64_t r = b.scalars[i];
    g1j R = (r == 1) ? P : jac_mul_u64_j(P, r);
    if (!jac_to_aff(R, out)) st = BLS_PK_IS_INFINITY;
  }
  st_g1a(b.pk_aff, b.n, i, out);
  pk_status[i] = (int8_t)st;
}

__global__ __launch_bounds__(WAVE) void k_sig_scale(PipelineBuffers b, uint32_t n_sets) {
  uint32_t i = blockIdx.x * WAVE + threadIdx.x;
  if (i >= n_sets) return;
  g2j R = jac_infinity<fp2>();
  if (b.status[i] == BLS_OK && !(b.flags[i] & SF_SIG_INF)) {
    g2a s = ld_g2a(b.sig_aff, b.n, i);
    uint64_t r = b.scalars[i];
    R = (r == 1) ? jac_from_aff(s) : jac_mul_u64(s, r);
  }
  st_g2j(b.rsig, b.n, i, R);
}

__global__ __launch_bounds__(WAVE) void k_miller_sets(PipelineBuffers b, uint32_t n_sets, const int8_t* pk_status) {
  uint32_t i = blockIdx.x * WAVE + threadIdx.x;
  if (i >= n_sets) return;
  fp12 f = fp12_one();
  if (b.status[i] == BLS_OK && pk_status[i] == BLS_OK && !(b.flags[b.n + i] & SF_H_INF)) {
    g1a P = ld_g1a(b.pk_aff, b.n, i);
    g2a Q = ld_g2a(b.h_aff, b.n, i);
    f = miller_loop(P, Q);
  }
  st_fp12(b.f, b.n, i, f);
}

__global__ __launch_bounds__(WAVE) void k_group_sig_miller(PipelineBuffers b, const uint32_t* group_first,
                                                           uint32_t n_groups, uint32_t* f_group,
                                                           const int8_t* pk_status) {
  uint32_t g = blockIdx.x * WAVE + threadIdx.x;
  if (g >= n_groups) return;
  g2j S = jac_infinity<fp2>();
  for (uint32_t i = group_first[g]; i < group_first[g + 1]; i++) {
    if (b.status[i] == BLS_OK && pk_status[i] == BLS_OK) S = jac_add(S, ld_g2j(b.rsig, b.n, i));
  }
  fp12 f = fp12_one();
  g2a Sa;
  if (jac_to_aff(S, Sa)) {
    g1a ng;
    ng.x = G1_GEN_X;
    ng.y = G1_NEG_GEN_Y;
    f = miller_loop(ng, Sa);
  }
  st_fp12(f_group, n_groups, g, f);
}

__global__ __launch_bounds__(WAVE) void k_group_finish(PipelineBuffers b, const uint32_t* group_first,
                                                       uint32_t n_groups, const uint32_t* f_group, uint8_t* group_ok) {
  uint32_t g = blockIdx.x * WAVE + threadIdx.x;
  if (g >= n_groups) return;
  fp12 f = ld_fp12(f_group, n_groups, g);
  for (uint32_t i = group_first[g]; i < group_first[g + 1]; i++) f = fp12_mul(f, ld_fp12(b.f, b.n, i));
  group_ok[g] = fp12_is_one(final_exponentiation(f)) ? 1 : 0;
}

__global__ __launch_bounds__(WAVE) void k_pk_table_fill(const uint8_t* pk96, uint32_t n, uint32_t* table_dst,
                                                        int8_t* status) {
  uint32_t i = blockIdx.x * WAVE + threadIdx.x;
  if (i >= n) return;
  uint8_t raw[96];
  for (int k = 0; k < 96; k++) raw[k] = pk96[(size_t)i * 96 + k];
  g1a a;
  bool inf = false;
  int st = pk_decode96(raw, a, inf);
  if (st == BLS_OK && inf) st = BLS_PK_IS_INFINITY;
  uint32_t* dst = table_dst + (size_t)i * W_PKTAB;
  for (int l = 0; l < BLS_NL; l++) {
    dst[l] = st == BLS_OK ? a.x.l[l] : 0;
    dst[BLS_NL + l] = st == BLS_OK ? a.y.l[l] : 0;
  }
  dst[2 * BLS_NL] = 0;
  dst[2 * BLS_NL + 1] = 0;
  dst[2 * BLS_NL + 2] = 0;
  dst[2 * BLS_NL + 3] = 0;
  status[i] = (int8_t)st;
}

// ------------------------------------------------------------------------------------- debug ops
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
    default:
      st = -2;
  }
  status[i] = st;
}

// ---------------------------------------------------------------------------------------- launchers
static inline dim3 grid_for(uint32_t n) { return dim3((n + WAVE - 1) / WAVE); }

void launch_sig_decode(const PipelineBuffers& b, uint32_t n, hipStream_t s) {
  if (n) hipLaunchKernelGGL(k_sig_decode, grid_for(n), dim3(WAVE), 0, s, b, n);
}
void launch_hash_to_g2(const PipelineBuffers& b, uint32_t n, hipStream_t s) {
  if (n) hipLaunchKernelGGL(k_hash_to_g2, grid_for(n), dim3(WAVE), 0, s, b, n);
}
void launch_pk_aggregate(const PipelineBuffers& b, uint32_t n, hipStream_t s) {
  if (n) hipLaunchKernelGGL(k_pk_aggregate, dim3(n), dim3(WAVE), 0, s, b, n);
}
void launch_pk_finish(const PipelineBuffers& b, uint32_t n, hipStream_t s) {
  // pk status lives right after the set status array (runtime allocates 2 * stride bytes)
  if (n) hipLaunchKernelGGL(k_pk_finish, grid_for(n), dim3(WAVE), 0, s, b, n, b.status + b.n);
}
void launch_sig_scale(const PipelineBuffers& b, uint32_t n, hipStream_t s) {
  if (n) hipLaunchKernelGGL(k_sig_scale, grid_for(n), dim3(WAVE), 0, s, b, n);
}
void launch_miller_sets(const PipelineBuffers& b, uint32_t n, hipStream_t s) {
  if (n) hipLaunchKernelGGL(k_miller_sets, grid_for(n), dim3(WAVE), 0, s, b, n, (const int8_t*)(b.status + b.n));
}
void launch_group_sig_miller(const PipelineBuffers& b, const uint32_t* group_first, uint32_t ng, uint32_t* f_group,
                             hipStream_t s) {
  if (ng)
    hipLaunchKernelGGL(k_group_sig_miller, grid_for(ng), dim3(WAVE), 0, s, b, group_first, ng, f_group,
                       (const int8_t*)(b.status + b.n));
}
void launch_group_finish(const PipelineBuffers& b, const uint32_t* group_first, uint32_t ng, const uint32_t* f_group,
                         uint8_t* group_ok, hipStream_t s) {
  if (ng) hipLaunchKernelGGL(k_group_finish, grid_for(ng), dim3(WAVE), 0, s, b, group_first, ng, f_group, group_ok);
}
void launch_pk_table_fill(const uint8_t* pk96, uint32_t n, uint32_t* table_dst, int8_t* status, hipStream_t s) {
  if (n) hipLaunchKernelGGL(k_pk_table_fill, grid_for(n), dim3(WAVE), 0, s, pk96, n, table_dst, status);
}
void launch_debug_op(int op, uint32_t n, const uint8_t* in, uint32_t in_stride, uint8_t* out, uint32_t out_stride,
                     int32_t* status, hipStream_t s) {
  if (n) hipLaunchKernelGGL(k_debug_op, grid_for(n), dim3(WAVE), 0, s, op, n, in, in_stride, out, out_stride, status);
}
