// A4 PublicKey.aggregate over the device pubkey table, r_i * pk_i (A9), and the table upload decoder.
#include "k_common.hpp"

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
STAGE_KERNEL void k_pk_finish(PipelineBuffers b, uint32_t n_sets, int8_t* pk_status) {
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

static inline dim3 grid_for(uint32_t n) { return dim3((n + WAVE - 1) / WAVE); }

void launch_pk_aggregate(const PipelineBuffers& b, uint32_t n, hipStream_t s) {
  if (n) hipLaunchKernelGGL(k_pk_aggregate, dim3(n), dim3(WAVE), 0, s, b, n);
}
void launch_pk_finish(const PipelineBuffers& b, uint32_t n, hipStream_t s) {
  // pk status lives right after the set status array (runtime allocates 2 * stride bytes)
  if (n) hipLaunchKernelGGL(k_pk_finish, grid_for(n), dim3(WAVE), 0, s, b, n, b.status + b.n);
}
void launch_pk_table_fill(const uint8_t* pk96, uint32_t n, uint32_t* table_dst, int8_t* status, hipStream_t s) {
  if (n) hipLaunchKernelGGL(k_pk_table_fill, grid_for(n), dim3(WAVE), 0, s, pk96, n, table_dst, status);
}
