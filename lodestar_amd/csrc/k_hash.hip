// A11 hash_to_G2, one lane per DISTINCT signing root of the call (the runtime deduplicates messages: gossip
// attestations of one committee share AttestationData, reference chain/validation/attestation.ts:131-138).
// Two kernels around the maps' one field inversion, which is batched over the messages in between
// (k_inv.hip, Montgomery's simultaneous inversion): k_hash_prep (hash_to_field .. d = a0 a1, stored with
// N(d)) -> k_batch_inv(N(d)) -> k_hash_map (one SSWU map + isogeny per lane, two lanes per message) ->
// k_hash_clear (sum, cofactor clearing; Jacobian H(m) + N(z)) -> k_batch_inv(N(z)) -> k_h_affine.
#include "k_common.hpp"
#include "g2_coop.hpp"

#define W_HPREP (7 * 2 * W_FP)
#ifndef BLSGPU_HASH_PAIRS
#define BLSGPU_HASH_PAIRS 1
#endif


// Q = q0 + q1, cofactor clearing (RFC 9380 G.3); Jacobian out + N(z) for the batched affine conversion.  The
// clearing (clear_cofactor_g2_slots) keeps the base point of each [|z|] chain -- Q, then A - psi(Q) -- in this lane's
// LDS slot (word-major, conflict-free), re-read at the chain's five additions, and C in h_jac[u] until the end: no
// point stays in registers across a chain, and the re-reads never reach HBM.
STAGE_KERNEL_W(BLSGPU_WPE_HASH) void k_hash_clear(PipelineBuffers b) {
  __shared__ uint32_t base[W_G2J * WAVE];
  const uint32_t u = blockIdx.x * WAVE + threadIdx.x;
  if (u >= b.n_umsg) return;
  const uint32_t qs = 2 * b.nm, t = threadIdx.x;
  st_g2j(base, WAVE, t, jac_add(ld_g2j(b.h_q, qs, 2 * u), ld_g2j(b.h_q, qs, 2 * u + 1)));
  const g2j H = clear_cofactor_g2_slots(
      [&](int k) { return k == 2 ? ld_g2j(b.h_jac, b.nm, u) : ld_g2j(base, WAVE, opaque_u32(t)); },
      [&](int k, const g2j& v) {
        if (k == 2)
          st_g2j(b.h_jac, b.nm, u, v);
        else
          st_g2j(base, WAVE, t, v);  // slot 1 (A - psi Q) replaces slot 0 (Q): read into registers before
      });
  st_g2j(b.h_jac, b.nm, u, H);
  st_fp(b.h_norm, b.nm, u, 0, fp2_norm(H.z));
}

// The same clearing on lane pairs (fp2x.hpp): lane 2m + k holds coefficient k of every Fp2 coordinate of message m's
// points, so a lane carries half a point and the kernel runs two waves per SIMD without spills.  The chain bases live
// in this lane's LDS slot (its coefficients only), C in h_jac[m] (coefficient k in the words of c_k).
#ifndef BLSGPU_WPE_HASH2
#define BLSGPU_WPE_HASH2 2
#endif
// this lane's slot: coordinate c at words c * W_FP .. + 13
__device__ __forceinline__ g2jx ld_g2jx_slot(const uint32_t* s, uint32_t t) {
  g2jx r;
  r.x.v = ld_fp(s, WAVE, t, 0);
  r.y.v = ld_fp(s, WAVE, t, W_FP);
  r.z.v = ld_fp(s, WAVE, t, 2 * W_FP);
  return r;
}
__device__ __forceinline__ void st_g2jx_slot(uint32_t* s, uint32_t t, const g2jx& v) {
  st_fp(s, WAVE, t, 0, v.x.v);
  st_fp(s, WAVE, t, W_FP, v.y.v);
  st_fp(s, WAVE, t, 2 * W_FP, v.z.v);
}
STAGE_KERNEL_W(BLSGPU_WPE_HASH2) void k_hash_clear2(PipelineBuffers b) {
  __shared__ uint32_t base[3 * W_FP * WAVE];
  const uint32_t q = blockIdx.x * WAVE + threadIdx.x, u = q >> 1, k = q & 1;
  if (u >= b.n_umsg) return;  // per pair: both lanes of a message leave together
  const uint32_t qs = 2 * b.nm, t = threadIdx.x;
  st_g2jx_slot(base, t, jac_add(ld_g2jx(b.h_q, qs, 2 * u, k), ld_g2jx(b.h_q, qs, 2 * u + 1, k)));
  const g2jx H = clear_cofactor_slots<fp2x>(
      [&](int s) { return s == 2 ? ld_g2jx(b.h_jac, b.nm, u, k) : ld_g2jx_slot(base, opaque_u32(t)); },
      [&](int s, const g2jx& v) {
        if (s == 2)
          st_g2jx(b.h_jac, b.nm, u, k, v);
        else
          st_g2jx_slot(base, t, v);
      });
  st_g2jx(b.h_jac, b.nm, u, k, H);
  const fp nz = fp2x_norm(H.z);
  if (k == 0) st_fp(b.h_norm, b.nm, u, 0, nz);
}

// The same clearing for small runs, latency first: one 16-lane group per message (g2_coop.hpp), four per workgroup;
// the two [|z|] chains run as cooperative doublings and additions, and so do the six additions around them
// (q0 + q1; B = A - psi(Q); A - Q; psi^2(2Q) - psi(Q); C; H = C + D) -- the lane-serial work left on the group's
// lane 0 is psi, psi^2, one doubling and the operand moves.  HBM scratch per message: Q in h_q[2u], B in h_q[2u + 1],
// A and then A - Q and C in h_jac[u] (all written and read by lane 0 only).
#define HC_GROUPS (WAVE / G2C_LANES)
__global__ __launch_bounds__(WAVE) void k_hash_clear_coop(PipelineBuffers b) {
  __shared__ uint32_t lds[HC_GROUPS * G2C_WORDS];
  const uint32_t tg = threadIdx.x % G2C_LANES, grp = threadIdx.x / G2C_LANES;
  const uint32_t u = blockIdx.x * HC_GROUPS + grp;
  const bool on = u < b.n_umsg;
  uint32_t* g = lds + grp * G2C_WORDS;
  const uint32_t qs = 2 * b.nm;
  const bool l0 = tg == 0 && on;
  if (l0) {
    g2c_st_point(g, ld_g2j(b.h_q, qs, 2 * u));
    g2c_st_q(g, ld_g2j(b.h_q, qs, 2 * u + 1));
  }
  g2c_sync();
  g2c_add(g, tg, on);  // Q = q0 + q1
  if (l0) st_g2j(b.h_q, qs, 2 * u, g2c_ld_point(g));
  g2c_sync();
  // A = [|z|] Q
  g2c_mul_zabs(g, tg, on, [&] { return ld_g2j(b.h_q, qs, 2 * opaque_u32(u)); });
  if (l0) {
    st_g2j(b.h_jac, b.nm, u, g2c_ld_point(g));  // A
    g2c_st_q(g, jac_neg(g2_psi(ld_g2j(b.h_q, qs, 2 * u))));
  }
  g2c_sync();
  g2c_add(g, tg, on);  // B = A - psi(Q)
  if (l0) {
    st_g2j(b.h_q, qs, 2 * u + 1, g2c_ld_point(g));
    g2c_st_point(g, ld_g2j(b.h_jac, b.nm, u));
    g2c_st_q(g, jac_neg(ld_g2j(b.h_q, qs, 2 * u)));
  }
  g2c_sync();
  g2c_add(g, tg, on);  // A - Q
  if (l0) {
    st_g2j(b.h_jac, b.nm, u, g2c_ld_point(g));
    const g2j Q = ld_g2j(b.h_q, qs, 2 * u);
    g2c_st_point(g, g2_psi2(jac_dbl(Q)));
    g2c_st_q(g, jac_neg(g2_psi(Q)));
  }
  g2c_sync();
  g2c_add(g, tg, on);  // psi^2(2Q) - psi(Q)
  if (l0) g2c_st_q(g, ld_g2j(b.h_jac, b.nm, u));
  g2c_sync();
  g2c_add(g, tg, on);  // C = psi^2(2Q) - psi(Q) + A - Q
  if (l0) {
    st_g2j(b.h_jac, b.nm, u, g2c_ld_point(g));
    g2c_st_point(g, ld_g2j(b.h_q, qs, 2 * u + 1));
  }
  g2c_sync();
  // D = [|z|] B; H = C + D
  g2c_mul_zabs(g, tg, on, [&] { return ld_g2j(b.h_q, qs, 2 * opaque_u32(u) + 1); });
  if (l0) g2c_st_q(g, ld_g2j(b.h_jac, b.nm, u));
  g2c_sync();
  g2c_add(g, tg, on);
  if (l0) {
    const g2j H = g2c_ld_point(g);
    st_g2j(b.h_jac, b.nm, u, H);
    st_fp(b.h_norm, b.nm, u, 0, fp2_norm(H.z));
  }
}

static inline dim3 grid_for(uint32_t n) { return dim3((n + WAVE - 1) / WAVE); }

void launch_hash_to_g2(const PipelineBuffers& b, hipStream_t s, bool coop, bool exclusive) {
  if (!b.n_umsg) return;
  launch_hash_prep(b, s);
  launch_batch_inv(b.h_norm, b.nm, 0, b.inv_buf, b.n_umsg, s);
  launch_hash_map(b, b.inv_buf, s);
  if (coop)
    hipLaunchKernelGGL(k_hash_clear_coop, dim3((b.n_umsg + HC_GROUPS - 1) / HC_GROUPS), dim3(WAVE),
                       BLSGPU_EXCLUSIVE_SMALL && exclusive ? exclusive_cu_lds<k_hash_clear_coop>() : 0, s, b);
  else if (BLSGPU_HASH_PAIRS)
    hipLaunchKernelGGL(k_hash_clear2, grid_for(2 * b.n_umsg), dim3(WAVE), 0, s, b);
  else
    hipLaunchKernelGGL(k_hash_clear, grid_for(b.n_umsg), dim3(WAVE), 0, s, b);
}
