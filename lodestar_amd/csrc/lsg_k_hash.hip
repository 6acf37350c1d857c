// lsg_k_hash.hip -- hash_to_G2 kernels (RFC 9380 BLS12381G2_XMD:SHA-256_SSWU_RO_ with the POP
// DST, blst's Hash_to_G2 inside Pairing.mul_n_aggregate under
// packages/beacon-node/src/chain/bls/maybeBatch.ts:18,37) and the SSZ
// signing roots of SURVEY.md 8f(3) (util/signingRoot.ts:7-13).
//
//   k_expand_msg   expand_message_xmd(msg_i, DST, 256), one thread per set (SHA-256)
//   k_h2c_prep     hash_to_field -> u0, u1; norms N(tv1(u0)), N(tv1(u1)) for one batched inversion
//   k_h2c_map      SSWU (shared-norm square root) -> 3-isogeny, one per field element; Q0 + Q1
//   k_h2c_clear    clear_cofactor (psi form); N(Z) for the second batched inversion
//   k_h2c_affine   (X, Y) * conj(Z) / N(Z)
#include "lsg_kcommon.hpp"

// waves per SIMD for the SSWU map and the cofactor clearing: 2 (256 registers, some scratch)
// or 1 (512 registers, none)
#ifndef LSG_H2C_WAVES
#define LSG_H2C_WAVES 2
#endif

// expand_message_xmd(msg_i, DST, 256) (RFC 9380 5.3.1; oracle/hash_to_curve.py), one thread
// per message.  Each thread's SHA-256 block buffer lives in LDS, byte k of thread t at word
// (k / 4) * 64 + t (consecutive threads, consecutive banks): a byte appended is one LDS byte
// store, where a register array indexed by the byte count went to scratch (a read-modify-
// write per byte).  The Z_pad block is compressed without being written; b_i's 32-byte prefix
// is stored as words; the output goes to global memory as words.
struct ShaLds {
  uint32_t st[8];
  uint32_t n, total;
  uint8_t* blk;  // this thread's byte 0; byte k at blk[(k >> 2) * 256 + (k & 3)]
};
LSG_DEVI void shal_init(ShaLds& c) {
  const uint32_t iv[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                          0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};
#pragma unroll
  for (int i = 0; i < 8; i++) c.st[i] = iv[i];
  c.n = 0;
  c.total = 0;
}
LSG_DEVI void shal_flush(ShaLds& c) {
  uint32_t w[16];
  const uint32_t* wl = (const uint32_t*)c.blk;
#pragma unroll
  for (int k = 0; k < 16; k++) w[k] = __builtin_bswap32(wl[k * 64]);
  sha256_compress(c.st, w);
  c.n = 0;
}
LSG_DEVI void shal_byte(ShaLds& c, uint8_t v) {
  c.blk[(c.n >> 2) * 256 + (c.n & 3)] = v;
  c.n++;
  c.total++;
  if (c.n == 64) shal_flush(c);
}
// a big-endian word at a word-aligned position (c.n % 4 == 0)
LSG_DEVI void shal_word(ShaLds& c, uint32_t v) {
  ((uint32_t*)c.blk)[(c.n >> 2) * 64] = __builtin_bswap32(v);
  c.n += 4;
  c.total += 4;
  if (c.n == 64) shal_flush(c);
}
LSG_DEVI void shal_final(ShaLds& c, uint32_t* out8) {
  const uint32_t bits = c.total * 8;  // (messages < 2^29 bytes)
  shal_byte(c, 0x80);
  while (c.n & 3) shal_byte(c, 0);
  if (c.n > 56)
    while (c.n) shal_word(c, 0);
  while (c.n < 60) shal_word(c, 0);
  shal_word(c, bits);
#pragma unroll
  for (int i = 0; i < 8; i++) out8[i] = c.st[i];
}

// append len bytes from src (global memory or LDS): the loads of 16 bytes are issued before
// the first append, so a lone message pays one memory round trip per 16 bytes, not per byte
LSG_DEVI void shal_bytes(ShaLds& c, const uint8_t* src, uint32_t len) {
  uint32_t k = 0;
  for (; k + 16 <= len; k += 16) {
    uint8_t b[16];
#pragma unroll
    for (int j = 0; j < 16; j++) b[j] = src[k + j];
#pragma unroll
    for (int j = 0; j < 16; j++) shal_byte(c, b[j]);
  }
  for (; k < len; k++) shal_byte(c, src[k]);
}

__global__ void __launch_bounds__(64) k_expand_msg(int n, const uint8_t* __restrict__ msg,
                                                    const uint32_t* __restrict__ msg_off,
                                                    const uint32_t* __restrict__ msg_len,
                                                    const uint8_t* __restrict__ dst, uint32_t dst_len,
                                                    uint8_t* __restrict__ ub) {
  __shared__ uint32_t lds[16 * 64];
  __shared__ uint8_t s_dst[256];  // the DST (< 256 bytes, RFC 9380), appended nine times
  for (uint32_t k = threadIdx.x; k < dst_len; k += 64) s_dst[k] = dst[k];
  __syncthreads();
  const size_t i = gtid();
  if (i >= (size_t)n) return;
  ShaLds c;
  c.blk = (uint8_t*)(lds + threadIdx.x);
  shal_init(c);
  {  // Z_pad: one all-zero block
    uint32_t z[16];
#pragma unroll
    for (int k = 0; k < 16; k++) z[k] = 0;
    sha256_compress(c.st, z);
    c.total = 64;
  }
  const uint8_t* m = msg + msg_off[i];
  const uint32_t ml = msg_len[i];
  shal_bytes(c, m, ml);
  shal_byte(c, 1);  // l_i_b_str = 256 (2 bytes, big endian)
  shal_byte(c, 0);
  shal_byte(c, 0);  // I2OSP(0, 1)
  shal_bytes(c, s_dst, dst_len);
  shal_byte(c, (uint8_t)dst_len);
  uint32_t b0[8], bi[8];
  shal_final(c, b0);
  uint32_t* o = (uint32_t*)(ub + 256 * i);
  for (int r = 1; r <= 8; r++) {
    shal_init(c);
#pragma unroll
    for (int k = 0; k < 8; k++) shal_word(c, r == 1 ? b0[k] : (b0[k] ^ bi[k]));
    shal_byte(c, (uint8_t)r);
    shal_bytes(c, s_dst, dst_len);
    shal_byte(c, (uint8_t)dst_len);
    shal_final(c, bi);
#pragma unroll
    for (int k = 0; k < 8; k++) o[8 * (r - 1) + k] = __builtin_bswap32(bi[k]);
  }
}

// stage 1: u0, u1 = hash_to_field(expand_message_xmd); norms N(tv1(u0)), N(tv1(u1)) at slots
// 2i, 2i+1 for the batched inversion
struct h2c_u_t {
  fp2_t u0, u1;
};
static_assert(lane_words<h2c_u_t>() == lsgl::W_H2CU, "layout: hash_to_field");

__global__ void LSG_KERNEL_ATTR k_h2c_prep(int n, const uint8_t* __restrict__ ub, uint32_t* __restrict__ U,
                                           uint32_t* __restrict__ norms) {
  LANE_ITEM(n);
  (void)lead;
  const uint8_t* b = ub + 256 * item;
  h2c_u_t u;
  u.u0 = fp2_make(fp_from_be64_mod(b), fp_from_be64_mod(b + 64));
  u.u1 = fp2_make(fp_from_be64_mod(b + 128), fp_from_be64_mod(b + 192));
  lane_store(U, item, u);
  lane_store(norms, 2 * item, fp2_norm(sswu_tv1(u.u0)));
  lane_store(norms, 2 * item + 1, fp2_norm(sswu_tv1(u.u1)));
}

// stage 2: SSWU -> 3-isogeny for one field element per item (2n items: u0 and u1 of set i
// are items 2i, 2i + 1, adjacent lane pairs of one quad), then P_i = Q_2i + Q_2i+1 by the even
// item with its neighbour's point moved over by a DPP quad permutation.  One map per item
// holds no second point while the other is computed (both in one item spilled 1.2 KB per
// lane).
template <class T>
LSG_DEVI T quad_swap_pairs(const T& v) {  // lanes 4i, 4i + 1 <-> 4i + 2, 4i + 3
  constexpr int W = sizeof(T) / 4;
  uint32_t w[W];
  __builtin_memcpy(w, &v, sizeof(T));
#pragma unroll
  for (int k = 0; k < W; k++) w[k] = pdpp<0x4E>(w[k]);  // quad_perm [2, 3, 0, 1]
  T r;
  __builtin_memcpy(&r, w, sizeof(T));
  return r;
}
__global__ void LSG_KERNEL_ATTR_W(LSG_H2C_WAVES) k_h2c_map(int n2, const uint32_t* __restrict__ U, const uint32_t* __restrict__ ninv,
                                          uint32_t* __restrict__ Hp) {
  LANE_ITEM(n2);  // n2 is even: both items of a set are live or neither is
  (void)lead;
  const g2p_t q = iso_map3(map_to_curve_sswu_ni(lane_load<fp2_t>(U, item), lane_load<fp_t>(ninv, item)));
  const g2p_t o = quad_swap_pairs(q);
  if ((item & 1) == 0) lane_store(Hp, item >> 1, g2_add(q, o));
}

// stage 2b: clear_cofactor in place; zN_i = N(Z) (0 at infinity) for the batched inversion.
// The [x] chains take their base point from an LDS slot per lane and the partial sum waits in
// the item's own slot of Hp, so the chains hold only their accumulator.
__global__ void LSG_KERNEL_ATTR_W(LSG_H2C_WAVES) k_h2c_clear(int n, uint32_t* __restrict__ Hp, uint32_t* __restrict__ zN,
                                            uint8_t* __restrict__ hinf) {
  __shared__ uint32_t park[sizeof(g2p_t) / 4 * LSG_TPB];
  LANE_ITEM(n);
  lds_park(park, lane_load<g2p_t>(Hp, item));
  g2p_t q = clear_cofactor_g2_parked([&]() { return lds_unpark<g2p_t>(park); },
                                     [&](const g2p_t& v) { lds_park(park, v); },
                                     [&](const g2p_t& v) { lane_store(Hp, item, v); },
                                     [&]() { return lane_load<g2p_t>(Hp, item); });
  bool is_inf = proj_is_inf(q);
  lane_store(Hp, item, q);
  lane_store(zN, item, is_inf ? fp_zero() : fp2_norm(q.Z));
  if (lead) hinf[item] = is_inf ? 1 : 0;
}

// each set's hashed point from its message's (packages whose sets share messages hash every
// distinct message once)
__global__ void LSG_KERNEL_ATTR k_h2c_gather(int n, const uint32_t* __restrict__ mid, const uint32_t* __restrict__ Hm,
                                             const uint8_t* __restrict__ hinfm, uint32_t* __restrict__ H,
                                             uint8_t* __restrict__ hinf) {
  LANE_ITEM(n);
  const uint32_t m = mid[item];
  lane_store(H, item, lane_load<g2a_t>(Hm, m));
  if (lead) hinf[item] = hinfm[m];
}

// stage 3: H affine = (X, Y) * conj(Z) / N(Z)   (= proj_to_aff, 1/Z = conj(Z) / N(Z))
__global__ void LSG_KERNEL_ATTR k_h2c_affine(int n, const uint32_t* __restrict__ Hp, const uint32_t* __restrict__ ninv,
                                             const uint8_t* __restrict__ hinf, uint32_t* __restrict__ H) {
  LANE_ITEM(n);
  (void)lead;
  g2p_t q = lane_load<g2p_t>(Hp, item);
  g2a_t a;
  if (hinf[item]) {
    a.x = fp2_zero();
    a.y = fp2_zero();
  } else {
    fp2_t zi = fp2_inv_with_norm_inv(q.Z, lane_load<fp_t>(ninv, item));
    a.x = fp2_mul(q.X, zi);
    a.y = fp2_mul(q.Y, zi);
  }
  lane_store(H, item, a);
}

// ---- SSZ signing roots, one thread per object.  Chunks are 8 big-endian
// SHA-256 words; every node is SHA-256 of exactly 64 bytes, so its second block is the
// constant padding block of a 512-bit message.
LSG_INL void ssz_hash2(const uint32_t* a, const uint32_t* b, uint32_t* out) {
  uint32_t st[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                    0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};
  uint32_t blk[16];
  for (int k = 0; k < 8; k++) {
    blk[k] = a[k];
    blk[8 + k] = b[k];
  }
  sha256_compress(st, blk);
  for (int k = 0; k < 16; k++) blk[k] = 0;
  blk[0] = 0x80000000u;
  blk[15] = 512;
  sha256_compress(st, blk);
  for (int k = 0; k < 8; k++) out[k] = st[k];
}

// `len` (<= 32) bytes at p as a zero-padded SSZ chunk
LSG_INL void ssz_chunk(uint32_t* w, const uint8_t* p, int len) {
  for (int k = 0; k < 8; k++) {
    uint32_t v = 0;
    for (int j = 0; j < 4; j++) v = (v << 8) | (4 * k + j < len ? p[4 * k + j] : 0u);
    w[k] = v;
  }
}

LSG_INL void ssz_store(uint8_t* out, const uint32_t* w) { be_words_to_bytes(out, w, 8); }

// hash_tree_root(SigningData{objectRoot, domain}) (util/signingRoot.ts:7-13)
__global__ void __launch_bounds__(64) k_signing_root(int n, const uint8_t* __restrict__ roots,
                                                     const uint8_t* __restrict__ domains, uint32_t dstride,
                                                     uint8_t* __restrict__ out32) {
  size_t i = gtid();
  if (i >= (size_t)n) return;
  uint32_t r[8], d[8], o[8];
  ssz_chunk(r, roots + 32 * i, 32);
  ssz_chunk(d, domains + dstride * i, 32);
  ssz_hash2(r, d, o);
  ssz_store(out32 + 32 * i, o);
}

// getAttestationDataSigningRoot (signatureSets/indexedAttestation.ts:11-19) from the SSZ
// serialization of phase0.AttestationData (128 bytes: slot u64, index u64, beaconBlockRoot,
// source {epoch u64, root}, target {epoch u64, root}): 5 fields -> 8 leaves, 3 levels, then
// SigningData -- 10 node hashes per object
__global__ void __launch_bounds__(64) k_attestation_signing_root(int n, const uint8_t* __restrict__ data,
                                                                 const uint8_t* __restrict__ domains,
                                                                 uint32_t dstride, uint8_t* __restrict__ out32) {
  size_t i = gtid();
  if (i >= (size_t)n) return;
  const uint8_t* a = data + 128 * i;
  uint32_t l0[8], l1[8], l2[8], l3[8], l4[8], t[8], z[8], z1[8], h01[8], h23[8], h45[8];
  for (int k = 0; k < 8; k++) z[k] = 0;
  ssz_chunk(l0, a, 8);        // slot
  ssz_chunk(l1, a + 8, 8);    // index
  ssz_chunk(l2, a + 16, 32);  // beaconBlockRoot
  ssz_chunk(t, a + 48, 8);    // source = Checkpoint{epoch, root}
  ssz_chunk(l3, a + 56, 32);
  ssz_hash2(t, l3, l3);
  ssz_chunk(t, a + 88, 8);  // target
  ssz_chunk(l4, a + 96, 32);
  ssz_hash2(t, l4, l4);
  ssz_hash2(z, z, z1);  // leaves 5..7 are zero chunks
  ssz_hash2(l0, l1, h01);
  ssz_hash2(l2, l3, h23);
  ssz_hash2(l4, z, h45);
  ssz_hash2(h01, h23, h01);
  ssz_hash2(h45, z1, h45);
  ssz_hash2(h01, h45, t);  // AttestationData.hashTreeRoot
  ssz_chunk(z, domains + dstride * i, 32);
  ssz_hash2(t, z, t);
  ssz_store(out32 + 32 * i, t);
}

namespace lsgk {
hipError_t expand_msg(hipStream_t st, int n, const uint8_t* msg, const uint32_t* off, const uint32_t* len,
                      const uint8_t* dst, uint32_t dst_len, uint8_t* ub) {
  if (n <= 0) return hipSuccess;
  if (dst_len > 255) return hipErrorInvalidValue;  // the kernel's LDS copy (RFC 9380: DST < 256 bytes)
  hipLaunchKernelGGL(k_expand_msg, dim3((n + 63) / 64), dim3(64), 0, st, n, msg, off, len, dst, dst_len, ub);
  return hipGetLastError();
}
hipError_t h2c_prep(hipStream_t st, int n, const uint8_t* ub, uint32_t* U, uint32_t* norms) {
  LSG_LAUNCH_ITEMS(k_h2c_prep, n, st, n, ub, U, norms);
}
hipError_t h2c_map(hipStream_t st, int n, const uint32_t* U, const uint32_t* ninv, uint32_t* Hp) {
  LSG_LAUNCH_ITEMS(k_h2c_map, 2 * n, st, 2 * n, U, ninv, Hp);
}
hipError_t h2c_clear(hipStream_t st, int n, uint32_t* Hp, uint32_t* zN, uint8_t* hinf) {
  LSG_LAUNCH_ITEMS(k_h2c_clear, n, st, n, Hp, zN, hinf);
}
hipError_t h2c_gather(hipStream_t st, int n, const uint32_t* mid, const uint32_t* Hm, const uint8_t* hinfm, uint32_t* H,
                      uint8_t* hinf) {
  LSG_LAUNCH_ITEMS(k_h2c_gather, n, st, n, mid, Hm, hinfm, H, hinf);
}
hipError_t h2c_affine(hipStream_t st, int n, const uint32_t* Hp, const uint32_t* ninv, const uint8_t* hinf,
                      uint32_t* H) {
  LSG_LAUNCH_ITEMS(k_h2c_affine, n, st, n, Hp, ninv, hinf, H);
}
hipError_t signing_root(hipStream_t st, int n, const uint8_t* roots, const uint8_t* domains, uint32_t dstride,
                        uint8_t* out32) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_signing_root, dim3((n + 63) / 64), dim3(64), 0, st, n, roots, domains, dstride, out32);
  return hipGetLastError();
}
hipError_t attestation_signing_root(hipStream_t st, int n, const uint8_t* data, const uint8_t* domains,
                                    uint32_t dstride, uint8_t* out32) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_attestation_signing_root, dim3((n + 63) / 64), dim3(64), 0, st, n, data, domains, dstride,
                     out32);
  return hipGetLastError();
}
}  // namespace lsgk
