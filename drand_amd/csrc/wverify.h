// Wave-cooperative latency engine: one beacon verification per wave, every limb of every field
// element in its own lane. Layers: wv.h (lanes, DPP, LDS; host emulation), wfield.h (Fp / Fp2 in
// 25-bit limbs, dot products with one Montgomery reduction), wtower.h (Fp12 as six w-power
// coefficients), wcurve.h (G2 Jacobian), whash.h (hash-to-G2, G2 decompression), wpairing.h (Miller
// loop, final exponentiation). The batch engine (fp.h ... pairing.h, one lane per beacon) stays the
// throughput path; blsverify.cpp routes small batches here.
#pragma once
#include "wpairing.h"

namespace wv {

// Fp coordinate of the batch engine's G1 tables (12 x 32-bit words, Montgomery R = 2^392, < 2p; a
// wave-uniform pointer) as a pair duplicated into both halves, Montgomery R = 2^400
WVI F g1_coord(const uint32_t* w12) {
  const V l = lane_id(), k = l & 15u;
  const V bit = k * 25u, wi = bit >> 5, sh = bit & 31u;
  const V lo = gld(w12, sel(wi < 12u, wi, vsplat(11))), hi = gld(w12, sel(wi < 11u, wi + 1u, vsplat(11)));
  const V v = ((lo >> sh) | sel((sh == 0u) | (wi >= 11u), vsplat(0), hi << ((32u - sh) & 31u))) & M25;  // (sh == 0: discarded)
  const V limbs = sel((l & 16u) == 0u, v, vsplat(0));
  return mulp(mkF(limbs, 2.0), cst(WC_C408_DUP));  // x 2^392 -> x 2^400
}

// the affine G2 point as the batch engine stores it: 2 x 12 words per coordinate, Montgomery-392
// (x.c0, x.c1, y.c0, y.c1), written by lane 0 of the wave... every lane holds the strict raw words
WVI void fp2_to392_words(const F& a, uint32_t (&w)[2][12]) {
  const V r = canon_times(a, WC_C392_DUP);  // a 2^392 mod p, strict limbs
  for (int h = 0; h < 2; h++) {
    uint32_t limb[16];
    for (int k = 0; k < 16; k++) limb[k] = lane_val(r, 32 * h + k);
    for (int j = 0; j < 12; j++) {
      const int b = 32 * j, k = b / 25, s = b % 25;
      uint64_t v = (uint64_t)limb[k] >> s;
      if (k + 1 < 16) v |= (uint64_t)limb[k + 1] << (25 - s);
      if (k + 2 < 16) v |= (uint64_t)limb[k + 2] << (50 - s);
      w[h][j] = (uint32_t)v;
    }
  }
}

// chain.VerifyBeacon / VerifyRecovered of one item: sig = 96-byte compressed signature, b0 = its
// message's expand_message_xmd b_0, pk = the G1 key (x, y words in the batch engine's form, or
// pk_inf). Returns the reject class (curve.h REJ_*); the decoded sigma on success (sx, sy, s_inf).
WVI uint8_t verify_item(const uint8_t* sig, const uint32_t (&b0)[8], const uint32_t* pkx, const uint32_t* pky,
                        bool pk_inf, F& sx, F& sy, bool& s_inf) {
  const uint8_t cls = g2_decompress(sig, sx, sy, s_inf);
  if (cls != bls::REJ_OK) return cls;
  F hx, hy;
  const bool h_fin = hash_to_g2(b0, hx, hy);
  MPair pr[2];
  const bool active[2] = {h_fin && !pk_inf, !s_inf};
  if (active[0]) pr[0] = mpair(g1_coord(pkx), g1_coord(pky), hx, hy);
  if (active[1]) pr[1] = mpair(cst(WC_NEG_G1_X), cst(WC_NEG_G1_Y), sx, sy);
  if (!active[0] && !active[1]) return bls::REJ_OK;  // empty product = 1 (kilic Check [ext])
  const W12 f0 = miller_loop(pr, active);
  return final_exp_is_one(f0) ? bls::REJ_OK : bls::REJ_PAIRING;
}

}  // namespace wv
