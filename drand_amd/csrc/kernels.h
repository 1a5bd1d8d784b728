// Kernel launchers of the beacon-verification engine (host-callable, defined in k_*.hip).
// Stage pipeline for a batch of beacons (each stage one lane per beacon, SoA staging in HBM):
//   hash   : message derivation + hash-to-G2            -> H[i]  (affine, 4 Fp slots) + h_inf[i]
//   decomp : sigma decompression + psi subgroup check    -> S[i]  (affine, 4 Fp slots) + s_inf[i], cls[i]
//   miller : e(pk_i, H_i) * e(-g1, S_i) multi-Miller loop -> F[i]  (Fp12, 12 Fp slots)
//   fexp   : final exponentiation, == 1                  -> cls[i] (REJ_PAIRING on mismatch)
//   finish : verdict bitmap (ballot) + first bad index (atomicMin)
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace blsk {

constexpr int H_WORDS = 48;   // affine G2
constexpr int S_WORDS = 48;   // affine G2
constexpr int F_WORDS = 144;  // Fp12
constexpr int G1_WORDS = 24;  // affine G1 (x, y Montgomery), AoS entry in pk tables

// Chained beacons (chain.VerifyBeacon with prev = the previous round's signature): item i has
// round first_round + i; with s = (i + seg_phase) / seg_len its prev is seeds[s] (length seed0_len
// for s == 0, else 96) when i == 0 or (i + seg_phase) % seg_len == 0, otherwise sigs[i-1].
// seg_len = n gives one continuous chain. seg_phase (< seg_len) is the position of item 0 inside
// its segment: a shard that starts mid-segment passes its halo (the true previous signature) as
// seeds[0] and the following segment seeds as seeds[1..] (shard.py, bench.py --total-rounds).
struct ChainedSrc {
  const uint8_t* sigs;   // n x 96 (global, whole batch)
  const uint8_t* seeds;  // n_seg x 96 slots
  uint64_t first_round;
  uint64_t seg_len;
  uint32_t seed0_len;  // 32 (genesis GroupHash) or 96
  uint64_t seg_phase;  // 0 for the generator and every host-buffer entry point
};

// Every hash launcher takes Q: HQ_WORDS x cnt words of SoA staging between its three kernels.
constexpr int HQ_WORDS = 144;
void launch_hash_chained(const ChainedSrc& src, size_t base, size_t cnt, uint32_t* H, uint8_t* h_inf,
                         uint32_t* Q, hipStream_t st);
// chain.VerifyBeaconV2: msg = sha256(BE64(round)); rounds == nullptr -> first_round + base + i
void launch_hash_unchained(const uint64_t* rounds, uint64_t first_round, size_t base, size_t cnt, uint32_t* H,
                           uint8_t* h_inf, uint32_t* Q, hipStream_t st);
// arbitrary messages (Scheme.VerifyRecovered / VerifyPartial / Sign): msg i = msgs[off[i] .. off[i]+len[i])
void launch_hash_messages(const uint8_t* msgs, const uint64_t* off, const uint32_t* len, size_t cnt,
                          uint32_t* H, uint8_t* h_inf, uint32_t* Q, hipStream_t st);
// 96-byte compressed signatures at sigs + (base+i)*stride + offset
void launch_decompress_g2(const uint8_t* sigs, size_t stride, size_t offset, size_t base, size_t cnt, uint32_t* S,
                          uint8_t* s_inf, uint8_t* cls, hipStream_t st);
// pk for item i: pk_tab[pk_idx ? pk_idx[i] : 0] (G1_WORDS each) with pk_inf flags
// LN: line staging for `sub` beacons (MILLER_LINE_WORDS each); the chunk runs in sub-chunks of `sub`
// (the host passes the whole chunk: blsverify.cpp kLineSub)
constexpr int MILLER_LINE_WORDS = 68 * 2 * 6 * 12;
void launch_miller(const uint32_t* pk_tab, const uint8_t* pk_inf, const uint32_t* pk_idx, const uint32_t* H,
                   const uint8_t* h_inf, const uint32_t* S, const uint8_t* s_inf, const uint8_t* cls, size_t cnt,
                   uint32_t* F, uint32_t* LN, size_t sub, uint32_t* park, hipStream_t st);
// park: TRI_PARK_WORDS(sub) words of scratch for the 3-lane f pass (48 words per lane, 21 items per wave)
constexpr size_t TRI_PARK_WORDS(size_t items) { return 48 * 64 * ((items + 20) / 21); }
// F is clobbered; W = 3 * cnt * F_WORDS words of staging; out (optional, test hook): the
// exponentiated values (SoA, cnt * F_WORDS words)
// park: FEXP_PARK_WORDS(cnt) words of scratch for the 3-lane products' parked partial results
constexpr size_t FEXP_PARK_WORDS(size_t items) { return TRI_PARK_WORDS(items); }
void launch_final_exp(uint32_t* F, uint32_t* W, size_t cnt, uint8_t* cls, hipStream_t st, uint32_t* park,
                      uint32_t* out = nullptr);
// bitmap bit (base+i) = (cls[i] == 0); bitmap must cover whole 64-bit words;
// first_bad = label0 + min rejected index (label0 = first_round -> ROUND numbers)
void launch_finish(const uint8_t* cls, size_t base, size_t cnt, uint64_t* bitmap, unsigned long long* first_bad,
                   uint64_t label0, hipStream_t st);

// ---- latency path (k_lat.hip): one workgroup per item, the whole verification; writes cls[i] (REJ_*)
int lat_trace_read(uint64_t* out, int n, hipStream_t st);  // phase marks of item 0 (wteam.h WV_MARK)
int lat_trace_clear(hipStream_t st);
int lat_trace_enable(int on, hipStream_t st);  // the device-global flag WV_MARK tests (off by default)
extern int g_generic_chains_all;  // k_hash.hip: every lane through the generic cofactor / subgroup kernels (test hook)
// and, for the messages form with S != nullptr, the decoded sigma (H/S staging layout, stride cnt)
void launch_lat_chained(const ChainedSrc& src, size_t base, size_t cnt, const uint32_t* pk_tab, const uint8_t* pk_inf,
                        uint8_t* cls, hipStream_t st);
void launch_lat_unchained(const uint64_t* rounds, uint64_t first_round, const uint8_t* sigs, size_t base, size_t cnt,
                          const uint32_t* pk_tab, const uint8_t* pk_inf, uint8_t* cls, hipStream_t st);
void launch_lat_messages(const uint8_t* msgs, const uint64_t* off, const uint32_t* len, const uint8_t* sigs,
                         size_t stride, size_t offset, size_t cnt, const uint32_t* pk_tab, const uint8_t* pk_inf,
                         const uint32_t* pk_idx, uint8_t* cls, uint32_t* S, uint8_t* s_inf, hipStream_t st);

// ---- group / threshold / signing kernels (k_misc.hip)
// decompress cnt G1 points (48 B each) -> pk table entries + inf flags + reject class
void launch_decompress_g1(const uint8_t* in, size_t cnt, uint32_t* tab, uint8_t* inf, uint8_t* cls, hipStream_t st);
// PubPoly.Eval(idx[i]) over t commits (affine table, none at infinity assumed via inf flags)
void launch_pubpoly_eval(const uint32_t* commits, const uint8_t* commit_inf, uint32_t t, const uint32_t* idx,
                         size_t cnt, uint32_t* out_tab, uint8_t* out_inf, hipStream_t st);
// decode only on the latency engine (k_lat.hip; one two-wave workgroup per signature)
void launch_lat_decode(const uint8_t* sigs, size_t stride, size_t offset, size_t cnt, uint32_t* S, uint8_t* s_inf,
                       uint8_t* cls, hipStream_t st);
void launch_decompress_g2_only(const uint8_t* sigs, size_t stride, size_t offset, size_t cnt, uint32_t* S,
                               uint8_t* s_inf, uint8_t* cls, hipStream_t st);
// sum_i [lambda_i] S_i over the selected affine staging entries sel[i] (S in SoA of stride n_s),
// compressed to 96 bytes
// [lambda_i] S_sel[i] summed and compressed (k_latrec.hip, lane form); scratch >= t * 192 words
// saff (optional, k_lat.hip kLatSaffWords words): the sum's affine point for launch_lat_verify_pre
void launch_lat_recover(const uint32_t* S, size_t n_s, const uint8_t* s_inf, const uint32_t* sel,
                        const uint32_t* lambdas, uint32_t t, uint32_t* scratch, uint8_t* out96, hipStream_t st,
                        uint32_t* saff = nullptr);
// the fused round's VerifyRecovered in two launches (wvteam.h team_hash_key / verify_team_pre): H of
// message 0 of (msgs, off, len) and the Miller loop of (pk_tab[0], H) into hout, then the pairing
// check of the affine signature saff (launch_lat_recover) against it -> cls[0]
constexpr size_t kLatHoutWords = 448, kLatSaffWords = 192;
void launch_lat_hash_key(const uint8_t* msgs, const uint64_t* off, const uint32_t* len, const uint32_t* pk_tab,
                         const uint8_t* pk_inf, uint32_t* hout, hipStream_t st);
void launch_lat_verify_pre(const uint32_t* hout, const uint32_t* saff, uint8_t* cls, hipStream_t st);
// signatures: out + i*out_stride (+2 index prefix when index >= 0) = compress(sk * H(msg_i))
void launch_sign(const uint32_t* sk_words, int32_t index, const uint32_t* H, const uint8_t* h_inf, size_t cnt,
                 uint8_t* out, size_t out_stride, hipStream_t st);
// synthetic chained history (client/test/result/mock/result.go:98-132 recipe, per segment):
// fills sigs (n x 96) for rounds first_round .. first_round+n-1 with the ChainedSrc seed rule
void launch_gen_chained(const uint32_t* sk_words, const ChainedSrc& src, size_t n, uint8_t* sigs_out, hipStream_t st);

// ---- test hooks (k_misc.hip): raw field / group / pairing building blocks
void launch_test_fp_mul(const uint32_t* a, const uint32_t* b, size_t cnt, uint32_t* out, hipStream_t st);
void launch_test_pairing(const uint32_t* p_tab, const uint32_t* q_aff, size_t cnt, uint32_t* out_f, hipStream_t st);
void launch_test_unpack_g2(const uint32_t* H, size_t cnt, uint32_t* out, hipStream_t st);
// raw AoS Fp12 (144 words each, tower order) <-> Montgomery SoA staging
void launch_test_pack_fp12(const uint32_t* f, size_t cnt, uint32_t* F, hipStream_t st);
void launch_test_unpack_fp12(const uint32_t* F, size_t cnt, uint32_t* out, hipStream_t st);
// SoA F -> final_exponentiation(F) with the one-lane register form (pairing.h), SoA out
void launch_test_final_exp_ref(const uint32_t* F, size_t cnt, uint32_t* out, hipStream_t st);

}  // namespace blsk
