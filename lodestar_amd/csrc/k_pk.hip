// A4 PublicKey.aggregate (device pubkey table or per-key bytes), r_i * pk_i (A9), same-message unit sums,
// aggregate serialization (PublicKey.aggregate(...).toBytes()), KeyValidate and the table upload decoder.
#include "k_common.hpp"

#ifndef BLSGPU_PK_AGG_GROUPS
#define BLSGPU_PK_AGG_GROUPS 1
#endif
// One wave per set: strided partial sums of the set's pubkeys, then an LDS tree reduction.  Table mode reads
// pk_table[pk_index[k]]; bytes-aggregate mode decodes pk_bytes[96 k] (trusted keys, PublicKey.fromBytes
// without subgroup check, as the pool worker, worker.ts:110-116: an identity key adds nothing).  The first
// malformed key (lowest k) sets the set's aggregation status; an out-of-range table index sets DEVICE_ERROR
// (the runtime rejects such calls before launching, this is the kernel's own guard).
__global__ __launch_bounds__(WAVE) void k_pk_aggregate(PipelineBuffers b, uint32_t n_sets) {
  __shared__ uint32_t red[WAVE * W_G1J];
  __shared__ uint32_t err_k[WAVE];
  __shared__ int32_t err_c[WAVE];
  if (blockIdx.x >= n_sets) return;
  const uint32_t set = b.agg_sets ? b.agg_sets[blockIdx.x] : blockIdx.x;
  uint32_t lane = threadIdx.x;
  int8_t* agg_status = b.status + 2 * b.n;
  const uint32_t first = b.set_pk_first[set], last = b.set_pk_first[set + 1];
  g1j acc = jac_infinity<fp>();
  uint32_t my_err_k = 0xffffffffu;
  int my_err = 0;
  for (uint32_t k = first + lane; k < last; k += WAVE) {
    g1a q;
    if (b.pk_bytes) {
      uint8_t raw[96];
      const uint8_t* src = b.pk_bytes + (size_t)k * 96;
#pragma unroll
      for (int t = 0; t < 96; t++) raw[t] = src[t];
      bool inf = false;
      const int st = pk_decode96(raw, q, inf);
      if (st != BLS_OK) {
        if (my_err == 0) {
          my_err = st;
          my_err_k = k;
        }
        continue;
      }
      if (inf) continue;
    } else {
      const uint32_t idx = b.pk_index[k];
      if (idx >= b.pk_table_n) {
        if (my_err == 0) {
          my_err = BLS_DEVICE_ERROR;
          my_err_k = k;
        }
        continue;
      }
      q = ld_pktab(b.pk_table, idx);
    }
    acc = jac_add_aff(acc, q);
  }
  err_k[lane] = my_err_k;
  err_c[lane] = my_err;
  __syncthreads();
  if (lane == 0) {
    uint32_t bk = 0xffffffffu;
    int bc = 0;
    for (int l = 0; l < WAVE; l++)
      if (err_k[l] < bk) {
        bk = err_k[l];
        bc = err_c[l];
      }
    agg_status[set] = (int8_t)bc;
  }
  const uint32_t cnt = last - first;
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

// The same aggregation on L lanes per set (64 / L sets per wave; L = 8, 16 or 32), the partial sums reduced by an
// in-register butterfly (__shfl_xor inside the lane group, no LDS, no barrier): with many sets (C4: 32,768 sets of
// ~486 keys) a wave per set spent ~2x the useful additions in its 6-level tree and idle lanes; L is chosen so the
// launch still gives every SIMD a wave (launch_pk_aggregate).
BLS_INL fp fp_shfl_xor(const fp& x, int m) {
  fp r;
#pragma unroll
  for (int i = 0; i < BLS_NL; i++) r.l[i] = (uint32_t)__shfl_xor((int)x.l[i], m);
  return r;
}
template <int L>
__global__ __launch_bounds__(WAVE) __attribute__((amdgpu_waves_per_eu(2, 2))) void k_pk_aggregate_g(PipelineBuffers b, uint32_t n_sets) {
  const uint32_t q = blockIdx.x * WAVE + threadIdx.x, t = q % L;
  const uint32_t si = q / L;
  const bool on = si < n_sets;  // whole groups: n_sets * L lanes, groups never straddle a wave (L divides WAVE)
  const uint32_t set = on ? (b.agg_sets ? b.agg_sets[si] : si) : 0;
  const uint32_t first = on ? b.set_pk_first[set] : 0, last = on ? b.set_pk_first[set + 1] : 0;
  g1j acc = jac_infinity<fp>();
  uint32_t my_err_k = 0xffffffffu;
  int my_err = 0;
  for (uint32_t k = first + t; k < last; k += L) {
    g1a pt;
    if (b.pk_bytes) {
      uint8_t raw[96];
      const uint8_t* src = b.pk_bytes + (size_t)k * 96;
#pragma unroll
      for (int z = 0; z < 96; z++) raw[z] = src[z];
      bool inf = false;
      const int st = pk_decode96(raw, pt, inf);
      if (st != BLS_OK) {
        if (my_err == 0) {
          my_err = st;
          my_err_k = k;
        }
        continue;
      }
      if (inf) continue;
    } else {
      const uint32_t idx = b.pk_index[k];
      if (idx >= b.pk_table_n) {
        if (my_err == 0) {
          my_err = BLS_DEVICE_ERROR;
          my_err_k = k;
        }
        continue;
      }
      pt = ld_pktab(b.pk_table, idx);
    }
    acc = jac_add_aff(acc, pt);
  }
  // butterfly: after log2 L levels every lane of the group holds the sum (and the first error by key position)
#pragma unroll 1
  for (int m = L / 2; m >= 1; m >>= 1) {
    g1j o;
    o.x = fp_shfl_xor(acc.x, m);
    o.y = fp_shfl_xor(acc.y, m);
    o.z = fp_shfl_xor(acc.z, m);
    const uint32_t ok = (uint32_t)__shfl_xor((int)my_err_k, m);
    const int oc = __shfl_xor(my_err, m);
    if (ok < my_err_k) {
      my_err_k = ok;
      my_err = oc;
    }
    acc = jac_add(acc, o);
  }
  if (on && t == 0) {
    b.status[2 * b.n + set] = (int8_t)my_err;
    st_g1j(b.pk_jac, b.n, set, acc);
  }
}

// The set's (aggregated) public key as a Jacobian point + status.  Single-key bytes mode decodes pk_bytes;
// with pk_direct1 a one-key set of table / bytes-aggregate mode reads its key here (k_pk_aggregate skipped it:
// the aggregate of one key is that key, an identity key aggregates to the identity).
__device__ __forceinline__ int set_pubkey(const PipelineBuffers& b, uint32_t i, g1j& P) {
  const bool one = b.set_pk_first && b.pk_direct1 && b.set_pk_first[i + 1] - b.set_pk_first[i] == 1;
  if (one && !b.pk_bytes) {
    const uint32_t idx = b.pk_index[b.set_pk_first[i]];
    if (idx >= b.pk_table_n) return BLS_DEVICE_ERROR;
    P = jac_from_aff(ld_pktab(b.pk_table, idx));
    return BLS_OK;
  }
  if (b.pk_bytes && (!b.set_pk_first || one)) {
    uint8_t raw[96];
    const uint32_t k = b.set_pk_first ? b.set_pk_first[i] : i;
    const uint4* src = reinterpret_cast<const uint4*>(b.pk_bytes + (size_t)k * 96);
#pragma unroll
    for (int k = 0; k < 6; k++) {
      uint4 v = src[k];
      uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int j = 0; j < 16; j++) raw[16 * k + j] = (uint8_t)(w[j >> 2] >> (8 * (j & 3)));
    }
    g1a a;
    bool inf = false;
    int st = pk_decode96(raw, a, inf);
    if (st == BLS_OK && inf) st = BLS_PK_IS_INFINITY;
    if (st == BLS_OK) P = jac_from_aff(a);
    return st;
  }
  if (b.set_pk_first[i + 1] == b.set_pk_first[i]) return BLS_EMPTY_AGGREGATE;
  const int st = b.status[2 * b.n + i];
  if (st) return st;
  P = ld_g1j(b.pk_jac, b.n, i);
  return jac_is_inf(P) ? BLS_PK_IS_INFINITY : BLS_OK;
}

// r_i * pk_i, Jacobian, in place of the aggregate in pk_jac (the affine conversion is batched, k_inv.hip
// k_pk_affine, which also maps an infinite r_i pk_i to PK_IS_INFINITY).  pk statuses go to their own array
// (status[n, 2n)); the job mask gives them precedence over signature statuses because the reference
// deserializes pubkeys first (worker.ts:39).  A set with a pubkey error stores the identity (z = 0), which
// the batch inversion skips.
STAGE_KERNEL_W(BLSGPU_WPE_PK) void k_pk_finish(PipelineBuffers b, uint32_t n_sets, int8_t* pk_status) {
  uint32_t i = blockIdx.x * WAVE + threadIdx.x;
  if (i >= n_sets) return;
  g1j P;
  int st = set_pubkey(b, i, P);
  g1j R = jac_infinity<fp>();
  if (st == BLS_OK) {
    const uint64_t w = b.scalars[i];  // batch scalar word, 0 = r = 1 (CoreVerify)
    R = (w == 0) ? P : jac_mul_scalar_word(P, w, b.scal_tab, b.n, i);
  }
  st_g1j(b.pk_jac, b.n, i, R);
  pk_status[i] = (int8_t)st;
}

// Same-message merging: P_u = sum of r_i pk_i over the unit's included sets (lane per unit).
STAGE_KERNEL void k_unit_aggregate(PipelineBuffers b) {
  uint32_t u = blockIdx.x * WAVE + threadIdx.x;
  if (u >= b.n_units) return;
  const uint32_t a = b.unit_set_first[u], e = b.unit_set_first[u + 1];
  g1a out;
  out.x = fp_zero();
  out.y = fp_zero();
  bool ok = false;
  if (e - a == 1) {
    const uint32_t i = b.unit_sets[a];
    if (b.include[i]) {
      out = ld_g1a(b.pk_aff, b.n, i);
      ok = true;
    }
  } else {
    g1j acc = jac_infinity<fp>();
    for (uint32_t k = a; k < e; k++) {
      const uint32_t i = b.unit_sets[k];
      if (b.include[i]) acc = jac_add_aff(acc, ld_g1a(b.pk_aff, b.n, i));
    }
    ok = jac_to_aff(acc, out);  // the identity (all excluded) pairs to 1
  }
  st_g1a(b.unit_p, b.n, u, out);
  b.unit_ok[u] = ok ? 1 : 0;
}

// PublicKey.aggregate(pks).toBytes(): 96-byte uncompressed or 48-byte compressed, per set.  status[3n...]
// receives 0 / EMPTY_AGGREGATE / a key error; an aggregate equal to the identity encodes the identity.
__global__ __launch_bounds__(WAVE) void k_pk_serialize(PipelineBuffers b, uint32_t n_sets, uint8_t* out,
                                                       uint32_t out_len) {
  uint32_t i = blockIdx.x * WAVE + threadIdx.x;
  if (i >= n_sets) return;
  int st = b.set_pk_first[i + 1] == b.set_pk_first[i] ? BLS_EMPTY_AGGREGATE : b.status[2 * b.n + i];
  uint8_t buf[96];
  for (int k = 0; k < 96; k++) buf[k] = 0;
  if (st == BLS_OK) {
    g1a a;
    if (!jac_to_aff(ld_g1j(b.pk_jac, b.n, i), a)) {
      buf[0] = out_len == 48 ? 0xc0 : 0x40;
    } else if (out_len == 48) {
      g1a_compress(a, buf);
    } else {
      g1a_to_be96(a, buf);
    }
  }
  uint8_t* o = out + (size_t)i * out_len;
  for (uint32_t k = 0; k < out_len; k++) o[k] = buf[k];
  b.status[i] = (int8_t)st;
}

// KeyValidate of untrusted pubkeys, one lane per key -> 96-byte uncompressed + status.
__global__ __launch_bounds__(WAVE) void k_key_validate(const uint8_t* pks, uint32_t n, uint32_t pk_len, uint32_t stride,
                                                       uint8_t* out96, int8_t* status) {
  uint32_t i = blockIdx.x * WAVE + threadIdx.x;
  if (i >= n) return;
  uint8_t raw[96];
  const uint8_t* src = pks + (size_t)i * stride;
  for (uint32_t k = 0; k < 96; k++) raw[k] = k < pk_len ? src[k] : 0;
  g1a a;
  const int st = pk_key_validate(raw, pk_len, a);
  uint8_t buf[96];
  for (int k = 0; k < 96; k++) buf[k] = 0;
  if (st == BLS_OK) g1a_to_be96(a, buf);
  if (out96)
    for (int k = 0; k < 96; k++) out96[(size_t)i * 96 + k] = buf[k];
  status[i] = (int8_t)st;
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

// lanes per set: one wave per set while n sets leave SIMDs idle, else the fewest lanes (>= 8) that still give
// every SIMD a wave (n * L >= 65,536 lanes)
void launch_pk_aggregate(const PipelineBuffers& b, uint32_t n, hipStream_t s) {
  if (b.agg_sets) n = b.n_agg;
  if (!n) return;
  const uint32_t lanes = 1024 * WAVE;
  if ((uint64_t)n * 64 <= lanes || !BLSGPU_PK_AGG_GROUPS)
    hipLaunchKernelGGL(k_pk_aggregate, dim3(n), dim3(WAVE), 0, s, b, n);
  else if ((uint64_t)n * 32 <= 2 * lanes)
    hipLaunchKernelGGL(k_pk_aggregate_g<32>, dim3((n * 32 + WAVE - 1) / WAVE), dim3(WAVE), 0, s, b, n);
  else if ((uint64_t)n * 16 <= 2 * lanes)
    hipLaunchKernelGGL(k_pk_aggregate_g<16>, dim3((n * 16 + WAVE - 1) / WAVE), dim3(WAVE), 0, s, b, n);
  else
    hipLaunchKernelGGL(k_pk_aggregate_g<8>, dim3((n * 8 + WAVE - 1) / WAVE), dim3(WAVE), 0, s, b, n);
}
void launch_pk_finish(const PipelineBuffers& b, uint32_t n, hipStream_t s) {
  // pk status lives right after the set status array (runtime allocates 3 * stride bytes)
  if (n) hipLaunchKernelGGL(k_pk_finish, grid_for(n), dim3(WAVE), 0, s, b, n, b.status + b.n);
}
void launch_unit_aggregate(const PipelineBuffers& b, hipStream_t s) {
  if (b.n_units) hipLaunchKernelGGL(k_unit_aggregate, grid_for(b.n_units), dim3(WAVE), 0, s, b);
}
void launch_pk_serialize(const PipelineBuffers& b, uint32_t n, uint8_t* out, uint32_t out_len, hipStream_t s) {
  if (n) hipLaunchKernelGGL(k_pk_serialize, grid_for(n), dim3(WAVE), 0, s, b, n, out, out_len);
}
void launch_key_validate(const uint8_t* pks, uint32_t n, uint32_t pk_len, uint32_t stride, uint8_t* out96,
                         int8_t* status, hipStream_t s) {
  if (n) hipLaunchKernelGGL(k_key_validate, grid_for(n), dim3(WAVE), 0, s, pks, n, pk_len, stride, out96, status);
}
void launch_pk_table_fill(const uint8_t* pk96, uint32_t n, uint32_t* table_dst, int8_t* status, hipStream_t s) {
  if (n) hipLaunchKernelGGL(k_pk_table_fill, grid_for(n), dim3(WAVE), 0, s, pk96, n, table_dst, status);
}
