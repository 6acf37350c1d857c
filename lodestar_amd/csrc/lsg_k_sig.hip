// lsg_k_sig.hip -- signature kernels: Signature.fromBytes(sig, affine, validate=true)
// (packages/beacon-node/src/chain/bls/maybeBatch.ts:23,36), the points each
// set adds to its group's RLC signature sum (blst mul_n_aggregate; 8a M4), G2 serialisation
// and the test/bench signer.
#include "lsg_kcommon.hpp"

__global__ void LSG_KERNEL_ATTR k_sig_decode(int n, const uint8_t* __restrict__ sig, const uint32_t* __restrict__ sig_len,
                                             uint32_t* __restrict__ sig_aff, uint8_t* __restrict__ inf,
                                             int32_t* __restrict__ err) {
  LANE_ITEM(n);
  uint32_t len = sig_len[item];
  g2a_t p;
  p.x = fp2_zero();
  p.y = fp2_zero();
  bool is_inf = false;
  int e;
  if (len == 96)
    e = g2_uncompress(p, is_inf, sig + 192 * item);
  else if (len == 192)
    e = g2_deserialize_uncompressed(p, is_inf, sig + 192 * item);
  else
    e = LSG_BLST_INVALID_SIZE;
  lane_store(sig_aff, item, p);
  if (lead) {
    inf[item] = is_inf ? 1 : 0;
    err[item] = e;
  }
}

// psi(P) == [x]P (Jacobian doubling chain, complete additions); the chain's base point waits
// in an LDS slot per lane, re-read at the five additions, instead of in spilled registers
__global__ void LSG_KERNEL_ATTR k_sig_subgroup(int n, const uint32_t* __restrict__ sig_aff,
                                               const uint8_t* __restrict__ inf, int32_t* __restrict__ err) {
  __shared__ uint32_t park[sizeof(g2a_t) / 4 * LSG_TPB];
  LANE_ITEM(n);
  if (err[item] != 0 || inf[item]) return;
  lds_park(park, lane_load<g2a_t>(sig_aff, item));
  bool ok = g2_in_group_get([&]() { return proj_from_aff(lds_unpark<g2a_t>(park)); });
  if (lead && !ok) err[item] = LSG_BLST_POINT_NOT_IN_GROUP;
}

// The point set i adds to its group's signature sum S_g = sum r_i sig_i: the identity for a
// set that cannot contribute (undecodable or infinite signature, infinite aggregated key: the
// verdict rules exclude such sets, lsg_host.hip), else sig_i (k_sig_proj: bucket MSM groups
// scale later) or [r_i] sig_i (k_sig_scale3: groups below the MSM threshold, sets whose mode
// byte is set).  Two kernels, so that the MSM path never carries the scaled path's window
// table.
LSG_DEVI bool sig_usable(size_t i, const uint8_t* inf, const int32_t* err, const uint8_t* pinf) {
  return err[i] == 0 && !inf[i] && !(pinf && pinf[i]);
}
__global__ void LSG_KERNEL_ATTR k_sig_proj(int n, const uint32_t* __restrict__ sig_aff, const uint8_t* __restrict__ inf,
                                           const int32_t* __restrict__ err, const uint8_t* __restrict__ pinf,
                                           uint32_t* __restrict__ out) {
  LANE_ITEM(n);
  (void)lead;
  g2p_t r = proj_inf<fp2_t>();
  if (sig_usable(item, inf, err, pinf)) r = proj_from_aff(lane_load<g2a_t>(sig_aff, item));
  lane_store(out, item, r);
}
// [r_i] sig_i with signed 3-bit windows (65 doublings + 22 additions, the window table in
// 512 registers at 1 wave per SIMD, no scratch; 4-bit windows with the table in scratch were
// measured slower: profiles/r03_*_scale3ab.json)
__global__ void LSG_KERNEL_ATTR_W(1) k_sig_scale3(int n, const uint32_t* __restrict__ sig_aff, const uint8_t* __restrict__ inf,
                                                  const int32_t* __restrict__ err, const uint8_t* __restrict__ pinf,
                                                  const uint64_t* __restrict__ rnd, const uint8_t* __restrict__ mode,
                                                  uint32_t* __restrict__ out) {
  LANE_ITEM(n);
  (void)lead;
  if (mode && !mode[item]) return;  // a set of an MSM group: k_sig_proj wrote its point
  g2p_t r = proj_inf<fp2_t>();
  if (sig_usable(item, inf, err, pinf)) {
    r = proj_from_aff(lane_load<g2a_t>(sig_aff, item));
    if (rnd[item] != 0) r = proj_mul_u64_s3(r, rnd[item]);  // r_i = 0: a set verified alone, not scaled
  }
  lane_store(out, item, r);
}

__global__ void LSG_KERNEL_ATTR k_g2a_to_bytes(int n, const uint32_t* __restrict__ pts, const uint8_t* __restrict__ inf,
                                               uint8_t* __restrict__ out) {
  LANE_ITEM(n);
  (void)lead;
  g2_serialize(out + 192 * item, lane_load<g2a_t>(pts, item), inf[item] != 0);
}

// projective G2 -> ZCash-compressed 96 bytes (Signature.toBytes(); the identity -> 0xc0 || 0^95)
__global__ void LSG_KERNEL_ATTR k_g2p_compress(int n, const uint32_t* __restrict__ pts, uint8_t* __restrict__ out96) {
  LANE_ITEM(n);
  (void)lead;
  g2p_t p = lane_load<g2p_t>(pts, item);
  bool is_inf = proj_is_inf(p);
  g2a_t a;
  if (is_inf) {
    a.x = fp2_zero();
    a.y = fp2_zero();
  } else {
    a = proj_to_aff(p);
  }
  g2_compress(out96 + 96 * item, a, is_inf);
}

// projective G2 (lane form) -> canonical 288-byte blobs for the row-backend group stages
__global__ void LSG_KERNEL_ATTR k_g2p_to_canon(int n, const uint32_t* __restrict__ in, uint8_t* __restrict__ out) {
  LANE_ITEM(n);
  (void)lead;
  g2p_to_canon_bytes(out + 288 * item, lane_load<g2p_t>(in, item));
}

// [k]P for a 256-bit big-endian scalar (test-data utilities only: signing, keygen)
template <class F>
__device__ proj_t<F> proj_mul_be256(const proj_t<F>& p, const uint8_t* k) {
  proj_t<F> acc = proj_inf<F>();
  for (int byte = 0; byte < 32; byte++) {
    uint32_t v = k[byte];
    for (int b = 7; b >= 0; b--) {
      acc = gdbl(acc);
      proj_t<F> s = gadd(acc, p);
      bool bit = (v >> b) & 1u;
      acc.X = fselect(bit, s.X, acc.X);
      acc.Y = fselect(bit, s.Y, acc.Y);
      acc.Z = fselect(bit, s.Z, acc.Z);
    }
  }
  return acc;
}

// sig_i = [sk_i] H(m_i), ZCash-compressed (bench/test input generation; not on the verify path)
__global__ void LSG_KERNEL_ATTR k_sign(int n, const uint8_t* __restrict__ sks, const uint32_t* __restrict__ H,
                                       uint8_t* __restrict__ out96) {
  LANE_ITEM(n);
  (void)lead;
  g2p_t s = proj_mul_be256(proj_from_aff(lane_load<g2a_t>(H, item)), sks + 32 * item);
  bool is_inf = proj_is_inf(s);
  g2a_t a;
  if (is_inf) {
    a.x = fp2_zero();
    a.y = fp2_zero();
  } else {
    a = proj_to_aff(s);
  }
  g2_compress(out96 + 96 * item, a, is_inf);
}

namespace lsgk {
hipError_t sig_decode(hipStream_t st, int n, const uint8_t* sig, const uint32_t* sig_len, uint32_t* sig_aff,
                      uint8_t* inf, int32_t* err) {
  LSG_LAUNCH_ITEMS(k_sig_decode, n, st, n, sig, sig_len, sig_aff, inf, err);
}
hipError_t sig_subgroup(hipStream_t st, int n, const uint32_t* sig_aff, const uint8_t* inf, int32_t* err) {
  LSG_LAUNCH_ITEMS(k_sig_subgroup, n, st, n, sig_aff, inf, err);
}
hipError_t sig_prep(hipStream_t st, int n, const uint32_t* sig_aff, const uint8_t* inf, const int32_t* err,
                    const uint8_t* pinf, const uint64_t* rnd, const uint8_t* mode, uint32_t* out) {
  if (n <= 0) return hipSuccess;
  if (!rnd || mode) {  // unscaled points for every set (mode: the scaled sets are overwritten next)
    hipLaunchKernelGGL(k_sig_proj, dim3(lane_blocks((size_t)n)), dim3(LSG_TPB), 0, st, n, sig_aff, inf, err, pinf, out);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || !rnd) return e;
  }
  return sig_scale_only(st, n, sig_aff, inf, err, pinf, rnd, mode, out);
}
hipError_t sig_scale_only(hipStream_t st, int n, const uint32_t* sig_aff, const uint8_t* inf, const int32_t* err,
                          const uint8_t* pinf, const uint64_t* rnd, const uint8_t* mode, uint32_t* out) {
  LSG_LAUNCH_ITEMS(k_sig_scale3, n, st, n, sig_aff, inf, err, pinf, rnd, mode, out);
}
hipError_t g2a_to_bytes(hipStream_t st, int n, const uint32_t* pts, const uint8_t* inf, uint8_t* out192) {
  LSG_LAUNCH_ITEMS(k_g2a_to_bytes, n, st, n, pts, inf, out192);
}
hipError_t g2p_compress(hipStream_t st, int n, const uint32_t* pts, uint8_t* out96) {
  LSG_LAUNCH_ITEMS(k_g2p_compress, n, st, n, pts, out96);
}
hipError_t g2p_to_canon(hipStream_t st, int n, const uint32_t* pts, uint8_t* out288) {
  LSG_LAUNCH_ITEMS(k_g2p_to_canon, n, st, n, pts, out288);
}
hipError_t sign(hipStream_t st, int n, const uint8_t* sks, const uint32_t* H, uint8_t* out96) {
  LSG_LAUNCH_ITEMS(k_sign, n, st, n, sks, H, out96);
}
}  // namespace lsgk
