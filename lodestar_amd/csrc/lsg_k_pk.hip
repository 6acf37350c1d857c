// lsg_k_pk.hip -- public-key kernels: deserializeSet's PublicKey.fromBytes (multithread/
// worker.ts:108-114) and the resident pubkey table gather (8f(1)), batched
// KeyValidate (8f(2), block/processDeposit.ts:57-65), the RLC scaling [r_i] aggPK_i of blst
// mul_n_aggregate (8a M4) and G1 serialisation.
#include "lsg_kcommon.hpp"
namespace {
#include "lsg_inv.hpp"
}  // namespace

// pubkey -> projective G1 (infinity and undecodable keys become (0:1:0)).  A key given by
// index (len == LSG_PK_INDEX: the slot's first 4 bytes) is gathered from the resident table
// (tab, tab_ok: decoded keys of lsg_pubkey_table_set; tab_n indices).
__global__ void LSG_KERNEL_ATTR k_pk_decode(int n, const uint8_t* __restrict__ pk, uint32_t stride,
                                            const uint32_t* __restrict__ pk_len,
                                            uint32_t* __restrict__ pkp, int32_t* __restrict__ err,
                                            const uint32_t* __restrict__ tab, const uint8_t* __restrict__ tab_ok,
                                            uint32_t tab_n) {
  LANE_ITEM(n);
  uint32_t len = pk_len[item];
  g1p_t p = proj_inf<fp_t>();
  int e;
  if (len == LSG_PK_INDEX) {
    const uint8_t* b = pk + (size_t)stride * item;
    const uint32_t idx = (uint32_t)b[0] | ((uint32_t)b[1] << 8) | ((uint32_t)b[2] << 16) | ((uint32_t)b[3] << 24);
    const bool ok = idx < tab_n && tab_ok[idx];
    e = ok ? 0 : LSG_ERR_BAD_INDEX;
    if (ok) p = lane_load<g1p_t>(tab, idx);
  } else {
    g1a_t a;
    a.x = fp_zero();
    a.y = fp_zero();
    bool is_inf = false;
    e = (len == 48 || len == 96) ? g1_deserialize(a, is_inf, pk + (size_t)stride * item, (int)len) : LSG_BLST_INVALID_SIZE;
    if (e == 0 && !is_inf) p = proj_from_aff(a);
  }
  lane_store(pkp, item, p);
  if (lead) err[item] = e;
}

// KeyValidate: decode, reject infinity and points outside G1; pts receives the key as a
// projective point (the identity for rejected keys); keys sit in 96-byte slots
__global__ void LSG_KERNEL_ATTR k_pk_validate(int n, const uint8_t* __restrict__ pk, uint32_t len,
                                              uint32_t* __restrict__ pts, int32_t* __restrict__ err) {
  LANE_ITEM(n);
  g1a_t a;
  a.x = fp_zero();
  a.y = fp_zero();
  bool is_inf = false;
  int e = g1_deserialize(a, is_inf, pk + 96 * item, (int)len);
  if (e == 0 && is_inf) e = LSG_BLST_PK_IS_INFINITY;
  const g1p_t p = e == 0 ? proj_from_aff(a) : proj_inf<fp_t>();
  if (e == 0 && !g1_in_group(p)) e = LSG_BLST_POINT_NOT_IN_GROUP;
  lane_store(pts, item, e == 0 ? p : proj_inf<fp_t>());
  if (lead) err[item] = e;
}

// P_i = [r_i] agg_i, projective (r_i == 0: no scaling); zP_i = its Z (0 at infinity) for the
// batched inversion; pinf = aggregate is infinity
__global__ void LSG_KERNEL_ATTR k_pk_scale(int n, const uint32_t* __restrict__ agg, const uint64_t* __restrict__ rnd,
                                           uint32_t* __restrict__ Pp, uint32_t* __restrict__ zP,
                                           uint8_t* __restrict__ pinf) {
  LANE_ITEM(n);
  g1p_t acc = lane_load<g1p_t>(agg, item);
  uint64_t r = rnd[item];
  bool is_inf = proj_is_inf(acc);
  if (r != 0 && !is_inf) acc = proj_mul_u64_s3(acc, r);
  lane_store(Pp, item, acc);
  lane_store(zP, item, is_inf ? fp_zero() : acc.Z);
  if (lead) pinf[item] = is_inf ? 1 : 0;
}

// P_i affine = (X / Z, Y / Z) with 1/Z from the batched inversion
__global__ void LSG_KERNEL_ATTR k_pk_affine(int n, const uint32_t* __restrict__ Pp, const uint32_t* __restrict__ zinv,
                                            uint32_t* __restrict__ P) {
  LANE_ITEM(n);
  (void)lead;
  g1p_t p = lane_load<g1p_t>(Pp, item);
  fp_t zi = lane_load<fp_t>(zinv, item);
  g1a_t a;
  fp_mul2(a.x, a.y, p.X, zi, p.Y, zi);
  lane_store(P, item, a);
}

// One Miller pair per distinct message (lsg_host.hip msg_agg): the package group's scaled keys
// r_i pk_i, each masked to the identity when its set cannot contribute (the rule of the Miller
// kernels: a decode error or an infinite key), are summed per message by the segmented
// reduction; the sums go affine with one divstep inversion each (a few dozen messages).
__global__ void LSG_KERNEL_ATTR k_pk_mask(int n, const uint32_t* __restrict__ Pp, const int32_t* __restrict__ err,
                                          const uint8_t* __restrict__ pinf, uint32_t* __restrict__ out) {
  LANE_ITEM(n);
  (void)lead;
  g1p_t p = proj_inf<fp_t>();
  if (err[item] == 0 && !pinf[item]) p = lane_load<g1p_t>(Pp, item);
  lane_store(out, item, p);
}
__global__ void LSG_KERNEL_ATTR k_g1p_affine_inv(int n, const uint32_t* __restrict__ Pp, uint32_t* __restrict__ P,
                                                 uint8_t* __restrict__ pinf) {
  LANE_ITEM(n);
  const g1p_t p = lane_load<g1p_t>(Pp, item);
  const bool is_inf = proj_is_inf(p);
  const fp_t d = pair_inv_gcd(pair_canon(is_inf ? fp_one() : p.Z));  // (Z R)^-1 as an integer
  const fp_t zi = pair_mont_mul(d, fp_t(FP_RCUBE));                   // Z^-1 R
  g1a_t a;
  fp_mul2(a.x, a.y, p.X, zi, p.Y, zi);
  lane_store(P, item, a);
  if (lead) pinf[item] = is_inf ? 1 : 0;
}

__global__ void LSG_KERNEL_ATTR k_g1p_to_bytes(int n, const uint32_t* __restrict__ pts, uint8_t* __restrict__ out) {
  LANE_ITEM(n);
  (void)lead;
  g1p_t p = lane_load<g1p_t>(pts, item);
  bool is_inf = proj_is_inf(p);
  g1a_t a;
  if (is_inf) {
    a.x = fp_zero();
    a.y = fp_zero();
  } else {
    a = proj_to_aff(p);
  }
  g1_serialize(out + 96 * item, a, is_inf);
}

// pk_i = [sk_i] G1, uncompressed 96 bytes (bench/test input generation; double-and-add)
__global__ void LSG_KERNEL_ATTR k_sk_to_pk(int n, const uint8_t* __restrict__ sks, uint8_t* __restrict__ out96) {
  LANE_ITEM(n);
  (void)lead;
  g1a_t g;
  g.x = fp_t(G1_GEN_X);
  g.y = fp_t(G1_GEN_Y);
  const g1p_t base = proj_from_aff(g);
  g1p_t acc = proj_inf<fp_t>();
  const uint8_t* k = sks + 32 * item;
  for (int byte = 0; byte < 32; byte++) {
    uint32_t v = k[byte];
    for (int b = 7; b >= 0; b--) {
      acc = g1_dbl(acc);
      g1p_t s = g1_add(acc, base);
      bool bit = (v >> b) & 1u;
      acc.X = fp_select(bit, s.X, acc.X);
      acc.Y = fp_select(bit, s.Y, acc.Y);
      acc.Z = fp_select(bit, s.Z, acc.Z);
    }
  }
  bool is_inf = proj_is_inf(acc);
  g1a_t a;
  if (is_inf) {
    a.x = fp_zero();
    a.y = fp_zero();
  } else {
    a = proj_to_aff(acc);
  }
  g1_serialize(out96 + 96 * item, a, is_inf);
}

namespace lsgk {
hipError_t pk_decode(hipStream_t st, int n, const uint8_t* pk, uint32_t stride, const uint32_t* pk_len, uint32_t* pts,
                     int32_t* err, const uint32_t* tab, const uint8_t* tab_ok, uint32_t tab_n) {
  LSG_LAUNCH_ITEMS(k_pk_decode, n, st, n, pk, stride, pk_len, pts, err, tab, tab_ok, tab_n);
}
hipError_t pk_validate(hipStream_t st, int n, const uint8_t* pk, uint32_t len, uint32_t* pts, int32_t* err) {
  LSG_LAUNCH_ITEMS(k_pk_validate, n, st, n, pk, len, pts, err);
}
hipError_t pk_scale(hipStream_t st, int n, const uint32_t* agg, const uint64_t* rnd, uint32_t* Pp, uint32_t* zP,
                    uint8_t* pinf) {
  LSG_LAUNCH_ITEMS(k_pk_scale, n, st, n, agg, rnd, Pp, zP, pinf);
}
hipError_t pk_affine(hipStream_t st, int n, const uint32_t* Pp, const uint32_t* zinv, uint32_t* P) {
  LSG_LAUNCH_ITEMS(k_pk_affine, n, st, n, Pp, zinv, P);
}
hipError_t pk_mask(hipStream_t st, int n, const uint32_t* Pp, const int32_t* err, const uint8_t* pinf, uint32_t* out) {
  LSG_LAUNCH_ITEMS(k_pk_mask, n, st, n, Pp, err, pinf, out);
}
hipError_t g1p_affine_inv(hipStream_t st, int n, const uint32_t* Pp, uint32_t* P, uint8_t* pinf) {
  LSG_LAUNCH_ITEMS(k_g1p_affine_inv, n, st, n, Pp, P, pinf);
}
hipError_t g1p_to_bytes(hipStream_t st, int n, const uint32_t* pts, uint8_t* out96) {
  LSG_LAUNCH_ITEMS(k_g1p_to_bytes, n, st, n, pts, out96);
}
hipError_t sk_to_pk(hipStream_t st, int n, const uint8_t* sks, uint8_t* out96) {
  LSG_LAUNCH_ITEMS(k_sk_to_pk, n, st, n, sks, out96);
}
}  // namespace lsgk
