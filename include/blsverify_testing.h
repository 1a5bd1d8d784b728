/*
 * blsverify_testing.h -- building-block entry points used only by the parity tests (tests/) to
 * check the device field and pairing arithmetic against the CPU oracle. Not part of the drop-in
 * boundary; exported by the same shared library.
 */
#ifndef DRAND_AMD_BLSVERIFY_TESTING_H
#define DRAND_AMD_BLSVERIFY_TESTING_H

#include "blsverify.h"

#ifdef __cplusplus
extern "C" {
#endif

/* out[i] = a[i] * b[i] mod p; 12 little-endian u32 limbs per element, canonical (< p) inputs. */
int blsv_test_fp_mul(blsv_ctx* ctx, const uint32_t* a, const uint32_t* b, size_t n, uint32_t* out);

/*
 * out_f[i] = e(P_i, Q_i)^3 (the engine's reduced pairing is the cube of the textbook value), as 144
 * u32 words: 12 Fp values (12 limbs each) in tower order c0.c0.{c0,c1}, c0.c1.{..}, c0.c2, c1.c0,
 * c1.c1, c1.c2. P: 24 words (x, y); Q: 48 words (x.c0, x.c1, y.c0, y.c1); raw (non-Montgomery).
 */
int blsv_test_pairing(blsv_ctx* ctx, const uint32_t* p, const uint32_t* q, size_t n, uint32_t* out_f);

/*
 * The production final-exponentiation stage (drand_amd/csrc/k_fexp.hip: the 3-lane hard part) and
 * the one-lane register form (pairing.h final_exponentiation) on the same n inputs f[i] (144 raw
 * words each, tower order as in blsv_test_pairing): out_pipeline[i] and out_ref[i] must agree.
 */
int blsv_test_final_exp(blsv_ctx* ctx, const uint32_t* f, size_t n, uint32_t* out_pipeline, uint32_t* out_ref);

/* out[i] = H(msg_i) as affine raw words (x.c0, x.c1, y.c0, y.c1; 48 words) + inf flag. */
int blsv_test_hash_to_g2(blsv_ctx* ctx, const uint8_t* msgs, const uint32_t* msg_lens, size_t n, uint32_t* out,
                         uint8_t* inf);

/*
 * on != 0: every hash's cofactor clearing and every decoded signature's subgroup check take the
 * generic path (k_hash.hip k_hash_cofactor_generic, k_decomp.hip k_subgroup_g2_generic: the formulas
 * with every exceptional case) instead of only the lanes the call-free chains flag; 0 restores
 * production. One process-global switch (all contexts), for the cross-check of both paths.
 */
int blsv_test_generic_chains(blsv_ctx* ctx, int on);

/*
 * Speculative recoveries of this context (blsv_aggregate / blsv_aggregate_round on the latency path):
 * hits = kept (the partials' verdicts left the speculated share selection unchanged), misses =
 * recomputed after a selected share failed.
 */
int blsv_test_spec_stats(blsv_ctx* ctx, uint64_t* hits, uint64_t* misses);

/*
 * Reconfigures a service's dispatcher context for the tests of its multi-pass and overflow paths
 * (waits until no batch is running): chunk != 0 sets the pipeline pass size to chunk items rounded up
 * to 64 (below the public floor kMinChunk on purpose, so that a small burst spans several passes);
 * lat_max sets the latency-path cutover (SIZE_MAX keeps it; 0 = batch pipeline only); arena_entries
 * != 0 caps the key arena (and empties it), so that a burst overflows it and runs as sub-batches.
 * *sub_launches (may be NULL) receives the number of device batches the service has run so far (a
 * coalesced batch split for the arena counts once per sub-batch). All three 0: only the count.
 */
int blsv_test_service_limits(blsv_service* svc, size_t chunk, size_t lat_max, size_t arena_entries,
                             uint64_t* sub_launches);

/*
 * Stage timing for bench.py's roofline: when enabled, every stage launch (0 hash, 1 decompress,
 * 2 miller, 3 final_exp, 4 finish, 5 lat = a whole batch on the latency path) is bracketed by HIP
 * events on its launch stream. blsv_profile_read waits for the recorded events, writes per-stage
 * summed milliseconds, launch counts and items processed (arrays of nstages), clears the records and
 * returns the number of stages the engine defines (6).
 */
int blsv_profile_enable(blsv_ctx* ctx, int on);
/*
 * Phase marks of the latency path (k_lat.hip). Off by default: blsv_lat_trace_enable(ctx, 1) turns
 * them on for the whole device (one device-global flag; production launches never stamp), 0 off again.
 * While on, item 0 of each latency launch stamps the device wall clock at up to 16 marks of wvteam.h
 * verify_team (0 start, 1 hash done, 2 signature decoded, 3 signature pair's Miller loop done, 4 phase
 * A joined, 5 key pair's Miller loop done, 6 Miller product ready, 7 final exponentiation done, 8/9
 * first exponentiation by |x| start/end, 10-13 hash: xmd done, both SSWU maps done, isogeny + addition
 * done, cofactor cleared, 14 signature's square root done (before its subgroup check), 15 signature
 * subgroup check done). The marks are one device-global array: blsv_lat_trace waits for the whole
 * device (every stream of every context) before it copies n marks (0 = never stamped) into ticks,
 * the clock rate into *ticks_per_us, and zeroes the marks when clear != 0. Returns the number of
 * marks copied. Meant for one profiling process running one latency launch at a time.
 */
int blsv_lat_trace(blsv_ctx* ctx, uint64_t* ticks, int n, double* ticks_per_us, int clear);
int blsv_lat_trace_enable(blsv_ctx* ctx, int on);
int blsv_profile_read(blsv_ctx* ctx, double* ms, uint64_t* launches, uint64_t* items, int nstages);
/*
 * The Lagrange basis at 0 that blsv_recover / blsv_aggregate* interpolate with (kyber
 * share.RecoverCommit [ext]): lambda_i = prod_{j != i} x_j / (x_j - x_i) over Fr for x_i = idx[i] + 1,
 * written as t canonical 8-word little-endian scalars. Host arithmetic only (no device, no context):
 * BLSV_EINVAL for repeated indices.
 */
int blsv_test_lagrange(const uint32_t* idx, size_t t, uint32_t* out);

#ifdef __cplusplus
}
#endif

#endif
