// SHA-256, drand beacon messages and RFC 9380 hash-to-G2 on gfx950 (one lane per message).
//   chain.Message   = sha256(prevSig || BE64(round))   chain/beacon.go:103-108, chain/store.go:39-44
//   chain.MessageV2 = sha256(BE64(round))              chain/beacon.go:110-114
//   KyberG2.Hash    = hash_to_curve(msg, "BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_NUL_")  [ext]
// expand_message_xmd starts from the precomputed midstate of the all-zero Z_pad block, and its
// constant DST-tail blocks are generated words (bls_constants.h), so b0 costs 2 compressions and
// each b_i 2 (the second block of every b_i is identical).
#pragma once
#include "curve.h"

namespace bls {

DI uint32_t rotr32(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

DI void sha256_compress(uint32_t (&st)[8], const uint32_t (&blk)[16]) {
  uint32_t w[16];
#pragma unroll
  for (int i = 0; i < 16; i++) w[i] = blk[i];
  uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
#pragma unroll
  for (int t = 0; t < 64; t++) {
    uint32_t wt;
    if (t < 16) {
      wt = w[t];
    } else {
      uint32_t w15 = w[(t - 15) & 15], w2 = w[(t - 2) & 15];
      uint32_t s0 = rotr32(w15, 7) ^ rotr32(w15, 18) ^ (w15 >> 3);
      uint32_t s1 = rotr32(w2, 17) ^ rotr32(w2, 19) ^ (w2 >> 10);
      wt = w[t & 15] + s0 + w[(t - 7) & 15] + s1;
      w[t & 15] = wt;
    }
    uint32_t S1 = rotr32(e, 6) ^ rotr32(e, 11) ^ rotr32(e, 25);
    uint32_t ch = (e & f) ^ (~e & g);
    uint32_t t1 = h + S1 + ch + SHA256_K[t] + wt;
    uint32_t S0 = rotr32(a, 2) ^ rotr32(a, 13) ^ rotr32(a, 22);
    uint32_t mj = (a & b) ^ (a & c) ^ (b & c);
    uint32_t t2 = S0 + mj;
    h = g;
    g = f;
    f = e;
    e = d + t1;
    d = c;
    c = b;
    b = a;
    a = t1 + t2;
  }
  st[0] += a;
  st[1] += b;
  st[2] += c;
  st[3] += d;
  st[4] += e;
  st[5] += f;
  st[6] += g;
  st[7] += h;
}

// The same compression as straight VALU code for the latency engine's wave-uniform hashing (one
// wave runs ~20 compressions in a row on a lone verify's critical path): every rotation one
// v_alignbit, Ch and Maj one v_bfi_b32 each, the three-way xor of Sigma0/Sigma1 folded into the add
// that consumes it (v_xad_u32: (a ^ b) + c) -- 17 operations per round and 11 per schedule word
// against ~28 and ~14 from the plain form, whose uniform data the compiler otherwise keeps on the
// scalar unit with a lane read-back per rotation.
#ifdef BLS_HOST
DI void sha256_compress_fast(uint32_t (&st)[8], const uint32_t (&blk)[16]) { sha256_compress(st, blk); }
#else
DI uint32_t v_bfi(uint32_t m, uint32_t a, uint32_t b) {  // (m & a) | (~m & b)
  uint32_t r;
  asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "v"(m), "v"(a), "v"(b));
  return r;
}
DI uint32_t v_xad(uint32_t a, uint32_t b, uint32_t c) {  // (a ^ b) + c
  uint32_t r;
  asm("v_xad_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
DI uint32_t v_ror(uint32_t x, int n) { return __builtin_amdgcn_alignbit(x, x, n); }
DI void sha256_compress_fast(uint32_t (&st)[8], const uint32_t (&blk)[16]) {
  uint32_t w[16];
#pragma unroll
  for (int i = 0; i < 16; i++) w[i] = blk[i];
  uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
#pragma unroll
  for (int t = 0; t < 64; t++) {
    uint32_t wt;
    if (t < 16) {
      wt = w[t];
    } else {
      const uint32_t w15 = w[(t - 15) & 15], w2 = w[(t - 2) & 15];
      const uint32_t s0 = v_xad(v_ror(w15, 7) ^ v_ror(w15, 18), w15 >> 3, w[t & 15]);  // sigma0 + w[t-16]
      const uint32_t s1 = v_xad(v_ror(w2, 17) ^ v_ror(w2, 19), w2 >> 10, w[(t - 7) & 15]);
      wt = s0 + s1;
      w[t & 15] = wt;
    }
    const uint32_t t1 = v_xad(v_ror(e, 6) ^ v_ror(e, 11), v_ror(e, 25), v_bfi(e, f, g)) + h + wt + SHA256_K[t];
    const uint32_t t2 = v_xad(v_ror(a, 2) ^ v_ror(a, 13), v_ror(a, 22), v_bfi(a ^ b, c, b));  // Sigma0 + Maj
    h = g;
    g = f;
    f = e;
    e = d + t1;
    d = c;
    c = b;
    b = a;
    a = t1 + t2;
  }
  st[0] += a;
  st[1] += b;
  st[2] += c;
  st[3] += d;
  st[4] += e;
  st[5] += f;
  st[6] += g;
  st[7] += h;
}
#endif

// the batch kernels' choice (k_hash.hip): the plain form unless built with BLS_SHA_FAST_BATCH=1
#ifndef BLS_SHA_FAST_BATCH
#define BLS_SHA_FAST_BATCH 0
#endif
DI void sha256_compress_batch(uint32_t (&st)[8], const uint32_t (&blk)[16]) {
  if constexpr (BLS_SHA_FAST_BATCH) sha256_compress_fast(st, blk); else sha256_compress(st, blk);
}

DI void sha256_init(uint32_t (&st)[8]) {
#pragma unroll
  for (int i = 0; i < 8; i++) st[i] = SHA256_IV[i];
}

DI uint32_t load_be32(const uint8_t* p) {
  return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | (uint32_t)p[3];
}

// chain.Message(round, prev) for prev of 96 bytes (104-byte message, 2 blocks) or 32 bytes
// (40-byte message, 1 block: the round-1 genesis seed, chain/store.go:46-51, client/verify.go:122).
template <bool FAST = false>
DI void drand_message(uint32_t (&out)[8], const uint8_t* prev, int prev_len, uint64_t round) {
  auto compress = [](uint32_t(&s_)[8], const uint32_t(&b_)[16]) {
    if constexpr (FAST) sha256_compress_fast(s_, b_); else sha256_compress(s_, b_);
  };
  uint32_t st[8];
  sha256_init(st);
  uint32_t blk[16];
  const uint32_t rhi = (uint32_t)(round >> 32), rlo = (uint32_t)round;
  if (prev_len == 96) {
#pragma unroll
    for (int i = 0; i < 16; i++) blk[i] = load_be32(prev + 4 * i);
    compress(st, blk);
#pragma unroll
    for (int i = 0; i < 8; i++) blk[i] = load_be32(prev + 64 + 4 * i);
    blk[8] = rhi;
    blk[9] = rlo;
    blk[10] = 0x80000000u;
#pragma unroll
    for (int i = 11; i < 15; i++) blk[i] = 0;
    blk[15] = 104 * 8;
    compress(st, blk);
  } else {  // 32-byte prev
#pragma unroll
    for (int i = 0; i < 8; i++) blk[i] = load_be32(prev + 4 * i);
    blk[8] = rhi;
    blk[9] = rlo;
    blk[10] = 0x80000000u;
#pragma unroll
    for (int i = 11; i < 15; i++) blk[i] = 0;
    blk[15] = 40 * 8;
    compress(st, blk);
  }
#pragma unroll
  for (int i = 0; i < 8; i++) out[i] = st[i];
}

// chain.MessageV2(round)
template <bool FAST = false>
DI void drand_message_v2(uint32_t (&out)[8], uint64_t round) {
  auto compress = [](uint32_t(&s_)[8], const uint32_t(&b_)[16]) {
    if constexpr (FAST) sha256_compress_fast(s_, b_); else sha256_compress(s_, b_);
  };
  uint32_t st[8];
  sha256_init(st);
  uint32_t blk[16];
  blk[0] = (uint32_t)(round >> 32);
  blk[1] = (uint32_t)round;
  blk[2] = 0x80000000u;
#pragma unroll
  for (int i = 3; i < 15; i++) blk[i] = 0;
  blk[15] = 64;
  compress(st, blk);
#pragma unroll
  for (int i = 0; i < 8; i++) out[i] = st[i];
}

// big-endian 512-bit integer given as 16 BE words -> Fp (Montgomery): hi*2^256*R + lo*R mod p
DI fp fp_from_be512(const uint32_t* w) {
  fp hi = fp_zero(), lo = fp_zero();
#pragma unroll
  for (int i = 0; i < 8; i++) {
    hi.l[i] = w[7 - i];
    lo.l[i] = w[15 - i];
  }
  return fp_add(fp_mul(hi, fp_load_const(FP_2POW256_R2)), fp_mul(lo, fp_load_const(FP_R2)));
}

// b_1..b_8 of expand_message_xmd from b_0, then the four 64-byte field elements; each element is
// reduced as soon as its two blocks exist (16 words live instead of 64)
DI void xmd_tail_to_field(const uint32_t (&b0)[8], fp2& u0, fp2& u1) {
  uint32_t prev[8];
#pragma unroll
  for (int i = 0; i < 8; i++) prev[i] = 0;
  fp e[4];
#pragma unroll
  for (int k = 1; k <= 8; k++) {
    uint32_t st[8];
    sha256_init(st);
    uint32_t blk[16];
#pragma unroll
    for (int i = 0; i < 8; i++) {
      blk[i] = b0[i] ^ prev[i];
      blk[8 + i] = XMD_BI_A_TAIL[i];
    }
    blk[8] |= (uint32_t)k << 24;
    sha256_compress_batch(st, blk);
    sha256_compress_batch(st, XMD_BI_B);
    if (k & 1) {
#pragma unroll
      for (int i = 0; i < 8; i++) prev[i] = st[i];
    } else {
      uint32_t w[16];
#pragma unroll
      for (int i = 0; i < 8; i++) {
        w[i] = prev[i];
        w[8 + i] = st[i];
        prev[i] = st[i];
      }
      e[k / 2 - 1] = fp_from_be512(w);
    }
  }
  u0 = {e[0], e[1]};
  u1 = {e[2], e[3]};
}

// b_0 of expand_message_xmd for an arbitrary-length message (bytes), DST bytes from dst_rt
// (a runtime-indexable copy of DST): Z_pad || msg || 01 00 || 00 || DST || 2b
template <bool FAST = false>
DI void xmd_b0_bytes(uint32_t (&b0)[8], const uint8_t* msg, uint32_t len, const uint8_t* dst_rt) {
  auto compress = [](uint32_t(&s_)[8], const uint32_t(&b_)[16]) {
    if constexpr (FAST) sha256_compress_fast(s_, b_); else sha256_compress(s_, b_);
  };
  uint32_t st[8];
#pragma unroll
  for (int i = 0; i < 8; i++) st[i] = SHA256_ZPAD_MIDSTATE[i];
  const uint32_t L = len + 3 + DST_LEN + 1;
  const uint64_t total_bits = (uint64_t)(64 + L) * 8;
  const uint32_t nblk = (L + 9 + 63) / 64;
  for (uint32_t b = 0; b < nblk; b++) {
    uint32_t blk[16];
    for (int w = 0; w < 16; w++) {
      uint32_t v = 0;
      for (int k = 0; k < 4; k++) {
        uint32_t pos = b * 64 + w * 4 + k;
        uint32_t byte;
        if (pos < len) byte = msg[pos];
        else if (pos == len) byte = 0x01;
        else if (pos < len + 3) byte = 0x00;
        else if (pos < len + 3 + DST_LEN) byte = dst_rt[pos - len - 3];
        else if (pos == len + 3 + DST_LEN) byte = DST_LEN;
        else if (pos == L) byte = 0x80;
        else byte = 0;
        v = (v << 8) | byte;
      }
      blk[w] = v;
    }
    if (b == nblk - 1) {
      blk[14] = (uint32_t)(total_bits >> 32);
      blk[15] = (uint32_t)total_bits;
    }
    compress(st, blk);
  }
#pragma unroll
  for (int i = 0; i < 8; i++) b0[i] = st[i];
}

// hash_to_field(msg32, count = 2) over Fp2 with expand_message_xmd(SHA-256, len 256)
DI void hash_to_field_fp2(const uint32_t (&msg)[8], fp2& u0, fp2& u1) {
  uint32_t b0[8];
  {
    uint32_t st[8];
#pragma unroll
    for (int i = 0; i < 8; i++) st[i] = SHA256_ZPAD_MIDSTATE[i];
    uint32_t blk[16];
#pragma unroll
    for (int i = 0; i < 8; i++) {
      blk[i] = msg[i];
      blk[8 + i] = XMD_B0_A_TAIL[i];
    }
    sha256_compress_batch(st, blk);
    sha256_compress_batch(st, XMD_B0_B);
#pragma unroll
    for (int i = 0; i < 8; i++) b0[i] = st[i];
  }
  xmd_tail_to_field(b0, u0, u1);
}

// hash-to-G2 from field elements (map both, isogeny, add, clear cofactor)
DI g2j hash_field_to_g2(const fp2& u0, const fp2& u1);

// RFC 9380 §6.6.2 simplified SWU onto E2': y^2 = x^3 + A'x + B' (straight-line form, selects
// instead of branches so a wave never diverges on the is_square outcome).
//   tv1 = 1/(Z^2 u^4 + Z u^2) is supplied by the caller (both u of a hash share one inversion).
//   Square test and root of the norm come from ONE Fp exponentiation: gx2 = (Z u^2)^3 gx1, so
//   when N(gx1) is a non-residue, sqrt(N(gx2)) = N(u)^3 sqrt(-N(Z)^3) sqrt(-N(gx1)).
DI fp2 sswu_den(const fp2& u) {
  fp2 zu2 = fp2_mul(fp2_load_const(SSWU_Z), fp2_sqr(u));
  return fp2_add(fp2_sqr(zu2), zu2);
}

DI g2a map_to_curve_sswu(const fp2& u, const fp2& tv1) {
  const fp2 A = fp2_load_const(SSWU_A);
  const fp2 B = fp2_load_const(SSWU_B);
  fp2 zu2 = fp2_mul(fp2_load_const(SSWU_Z), fp2_sqr(u));
  fp2 x1 = fp2_mul(fp2_load_const(SSWU_MINUS_B_OVER_A), fp2_add(fp2_one(), tv1));
  x1 = fp2_select(fp2_is_zero(tv1), fp2_load_const(SSWU_B_OVER_ZA), x1);
  fp2 gx1 = fp2_add(fp2_mul(fp2_add(fp2_sqr(x1), A), x1), B);
  fp2 x2 = fp2_mul(zu2, x1);
  fp2 gx2 = fp2_mul(fp2_mul(fp2_sqr(zu2), zu2), gx1);
  bool sq1;
  fp r1 = fp_norm_root(fp2_norm(gx1), sq1);  // sqrt(N(gx1)) or sqrt(-N(gx1))
  fp nu = fp2_norm(u);
  fp r2 = fp_mul(fp_mul(fp_mul(fp_sqr(nu), nu), fp_load_const(SSWU_SQRT_MINUS_NZ3)), r1);
  fp2 x = fp2_select(sq1, x1, x2);
  fp2 gx = fp2_select(sq1, gx1, gx2);
  fp2 y = fp2_sqrt_with_norm_root(gx, fp_select(sq1, r1, r2));
  if (fp2_sgn0(u) != fp2_sgn0(y)) y = fp2_neg(y);
  return {x, y};
}

// RFC 9380 E.3 3-isogeny E2' -> E2, output in Jacobian coordinates without inversion:
// x = xn/xd, y = y' yn/yd  ->  Z = xd*yd, X = xn*xd*yd^2, Y = y'*yn*xd^3*yd^2
DI g2j iso_map_g2(const g2a& p) {
  const fp2 x = p.x;
  fp2 xn = fp2_load_const(ISO_XNUM[3]);
  xn = fp2_add(fp2_mul(xn, x), fp2_load_const(ISO_XNUM[2]));
  xn = fp2_add(fp2_mul(xn, x), fp2_load_const(ISO_XNUM[1]));
  xn = fp2_add(fp2_mul(xn, x), fp2_load_const(ISO_XNUM[0]));
  fp2 xd = fp2_add(x, fp2_load_const(ISO_XDEN[1]));  // monic
  xd = fp2_add(fp2_mul(xd, x), fp2_load_const(ISO_XDEN[0]));
  fp2 yn = fp2_load_const(ISO_YNUM[3]);
  yn = fp2_add(fp2_mul(yn, x), fp2_load_const(ISO_YNUM[2]));
  yn = fp2_add(fp2_mul(yn, x), fp2_load_const(ISO_YNUM[1]));
  yn = fp2_add(fp2_mul(yn, x), fp2_load_const(ISO_YNUM[0]));
  fp2 yd = fp2_add(x, fp2_load_const(ISO_YDEN[2]));  // monic
  yd = fp2_add(fp2_mul(yd, x), fp2_load_const(ISO_YDEN[1]));
  yd = fp2_add(fp2_mul(yd, x), fp2_load_const(ISO_YDEN[0]));
  fp2 Z = fp2_mul(xd, yd);
  fp2 yd2 = fp2_sqr(yd);
  fp2 X = fp2_mul(fp2_mul(xn, xd), yd2);
  fp2 xd3 = fp2_mul(fp2_sqr(xd), xd);
  fp2 Y = fp2_mul(fp2_mul(p.y, yn), fp2_mul(xd3, yd2));
  return {X, Y, Z};  // Z == 0 (exceptional isogeny kernel) gives the point at infinity
}

// one mapped point q = iso(map(u)) (Jacobian) with its own SSWU denominator inversion (a binary-GCD
// inversion is cheap, fp.h, so the two points of a hash are independent and can run in two lanes):
// tv = 1/(Z^2 u^4 + Z u^2), or 0 when that is 0 (RFC 9380 inv0)
DI g2j hash_field_to_q1(const fp2& u) {
  const fp2 d = sswu_den(u);
  const bool z = fp2_is_zero(d);
  const fp2 tv = fp2_select(z, fp2_zero(), fp2_inv(fp2_select(z, fp2_one(), d)));
  return iso_map_g2(map_to_curve_sswu(u, tv));
}

// the two mapped points q0 = iso(map(u0)), q1 = iso(map(u1)) in one lane: the exponentiation-heavy
// half of hash-to-G2 (one inversion shared by both SSWU denominators, four Fp exponentiations)
DI void hash_field_to_q(const fp2& u0, const fp2& u1, g2j& q0, g2j& q1) {
  // exact also when one of the denominators is 0: inv0(0) = 0
  fp2 d0 = sswu_den(u0), d1 = sswu_den(u1);
  const bool z0 = fp2_is_zero(d0), z1 = fp2_is_zero(d1);
  d0 = fp2_select(z0, fp2_one(), d0);
  d1 = fp2_select(z1, fp2_one(), d1);
  fp2 di = fp2_inv(fp2_mul(d0, d1));
  fp2 tv0 = fp2_select(z0, fp2_zero(), fp2_mul(d1, di));
  fp2 tv1 = fp2_select(z1, fp2_zero(), fp2_mul(d0, di));
  q0 = iso_map_g2(map_to_curve_sswu(u0, tv0));
  q1 = iso_map_g2(map_to_curve_sswu(u1, tv1));
}

DI g2j hash_field_to_g2(const fp2& u0, const fp2& u1) {
  g2j q0, q1;
  hash_field_to_q(u0, u1, q0, q1);
  return g2_clear_cofactor(jac_add(q0, q1));
}

// KyberG2.Hash(msg32): Jacobian result, cofactor cleared
DI g2j hash_to_g2(const uint32_t (&msg)[8]) {
  fp2 u0, u1;
  hash_to_field_fp2(msg, u0, u1);
  return hash_field_to_g2(u0, u1);
}

}  // namespace bls
