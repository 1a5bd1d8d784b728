/*
 * blsverify.h -- C ABI of the MI355X-native BLS12-381 beacon-verification engine.
 *
 * This is the drop-in boundary for drand's verification hot path. The reference
 * calls five methods on the package-level `key.Scheme` (tbls.NewThresholdSchemeOnG2(Pairing),
 * key/curve.go:31) plus the chain entry points built on it; each entry point below names the
 * reference interface it replaces. A cgo package (gpu/blsverify) binds these
 * symbols one-to-one.
 *
 * Conventions
 *  - All buffers are caller-owned host memory valid only for the duration of the call (cgo rules);
 *    the library copies into HBM and never retains caller pointers. The *_dev entry points take
 *    device pointers (HBM-resident batches, used by bench.py and multi-GPU sharding).
 *  - Return value: 0 = the call succeeded (per-item verdicts are in the outputs); < 0 =
 *    infrastructure error (bad arguments, HIP failure); details from blsv_last_error().
 *  - Accept/reject and recovered signature bytes are bit-exact with the reference kyber path;
 *    the optional reject_class output explains a reject (BLSV_REJ_*), error text is not graded.
 *  - Bitmaps: bit i (byte i/8, bit i%8, LSB first) = 1 iff item i verified.
 *  - first_bad: the ROUND number (chained/unchained) or the INDEX (message batches) of the first
 *    rejected item, UINT64_MAX when every item verified.
 *  - A context owns one HIP stream and is not thread-safe: one thread calls it at a time. For
 *    concurrent single-item callers use a blsv_service (thread-safe, coalesces concurrent calls into
 *    one launch; see the end of this header); for concurrent batch callers one context per thread,
 *    each with its chunk sized so that all of them fit in HBM (memory contract below).
 *
 * Latency contract (single-item and small callers: client.Get's per-round verify,
 * client/verify.go:185-207; the gossip validator, lp2p/client/validator.go:64; per-packet
 * VerifyPartial, chain/beacon/node.go:112,125; identity checks, key/keys.go:60-63)
 *  - A call with at most lat_max items (blsv_set_lat_max, default 1536) runs on the LATENCY path: one
 *    workgroup of eight waves per item, every limb of a field element in its own lane
 *    (drand_amd/csrc/k_lat.hip). Measured on MI355X (profiles/r06e_latency.json, warm): one
 *    VerifyRecovered 1.9 ms; blsv_aggregate of an n = 64 / t = 33 round (64 VerifyPartial +
 *    Recover + VerifyRecovered) 2.2 ms, blsv_aggregate_round V1 + V2 4.4 ms (the recovery and the
 *    verification of the shares the round would select if all verify run beside the partial
 *    verification -- H(msg) and the key pair's Miller loop from the start -- and are kept when the
 *    verdicts confirm that selection). Up to 256 items the time stays ~2.1 ms (every item has its
 *    own CU), then grows ~1.9 ms per further 256 items (profiles/r05za_latency_sweep.json).
 *  - Larger calls run on the BATCH pipeline (one lane per item, staged kernels): ~14 ms floor
 *    (14.1 ms at 64 items, 15.3 ms at 2,048: profiles/r05za_latency_sweep.json), then ~0.43 us per
 *    item (about 2.3 M items/s). Both paths give
 *    identical verdicts, reject classes and
 *    recovered bytes (tests/test_gpu_lat.py runs the same vectors through both).
 *  - The first call on a context also pays allocation and module load (~10-250 ms).
 */
#ifndef DRAND_AMD_BLSVERIFY_H
#define DRAND_AMD_BLSVERIFY_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct blsv_ctx blsv_ctx;

/* return codes */
#define BLSV_OK 0
#define BLSV_EINVAL (-1)
#define BLSV_EHIP (-2)
#define BLSV_ENOGROUP (-3)
#define BLSV_ENOTENOUGH (-4) /* Recover: fewer than t valid shares */

/* reject classes (per item) -- the order of kilic G2.FromCompressed's checks, then the pairing */
#define BLSV_REJ_OK 0
#define BLSV_REJ_LENGTH 1          /* wrong byte length (host-side)                      */
#define BLSV_REJ_FLAG 2            /* compression bit 0x80 clear                          */
#define BLSV_REJ_INF_NONZERO 3     /* infinity bit set but not exactly 0xc0 || 0...       */
#define BLSV_REJ_X_GE_P 4          /* a coordinate limb >= p                              */
#define BLSV_REJ_NOT_ON_CURVE 5    /* x^3 + b has no square root                          */
#define BLSV_REJ_NOT_IN_SUBGROUP 6 /* point not in the order-r subgroup                   */
#define BLSV_REJ_PAIRING 7         /* "bls: invalid signature" (pairing check failed)     */
#define BLSV_REJ_SHARE_INDEX 8     /* tbls share shorter than its 2-byte index prefix     */

#define BLSV_SIG_LEN 96
#define BLSV_PARTIAL_LEN 98
#define BLSV_PK_LEN 48

/* Library version string. */
const char* blsv_version(void);

/* Number of GPUs this process sees (0 when none or on a HIP error): one context per GPU for
 * blsv_verify_chained_multi. */
int blsv_device_count(void);

/* Create a context on HIP device `device`. */
int blsv_create(int device, blsv_ctx** out);
void blsv_destroy(blsv_ctx* ctx);
/* Last error message of this context ("" if none). */
const char* blsv_last_error(const blsv_ctx* ctx);

/*
 * Group state: the distributed public polynomial commitments (key.Share.PubPoly /
 * DistPublic.PubPoly, key/keys.go:235-241,316-324), t commitments of 48 bytes; the group public
 * key is commits[0] (DistPublic.Key(), chain.Info.PublicKey, chain/info.go:16-21). n is the group
 * size passed to Recover. A single-key chain is t = 1. Decoding follows kilic G1.FromCompressed
 * (chain/convert.go:15-18); returns BLSV_EINVAL if any commitment fails to decode.
 */
int blsv_set_group(blsv_ctx* ctx, const uint8_t* commits48, size_t t, size_t n);

/*
 * chain.VerifyBeacon (chain/beacon.go:87-92) over a contiguous chained range: beacon i has round
 * first_round + i, signature sigs96[i], and PreviousSig = prev0 (i == 0; 32 bytes = genesis seed
 * GroupHash at round 1, client/verify.go:122-124, or 96 bytes) or sigs96[i-1]. Replaces the serial
 * walk of client/verify.go:146-163 and chain/beacon/sync.go:100-119 with one batched call.
 * reject_class (optional, n bytes) receives BLSV_REJ_* per beacon.
 */
int blsv_verify_chained(blsv_ctx* ctx, uint64_t first_round, const uint8_t* prev0, size_t prev0_len,
                        const uint8_t* sigs96, size_t n, uint8_t* ok_bitmap, uint64_t* first_bad,
                        uint8_t* reject_class);

/*
 * blsv_verify_chained over SEVERAL contexts at once -- the multi-GPU shape of a Go host: one context
 * per GPU (ctxs[k] may sit on any device; each must hold the same group, set with blsv_set_group, and
 * appear once), one host thread per context. The range is split into n_ctx contiguous shards
 * (shard_counts[k] beacons each, summing to n; NULL = an even split, the first n % n_ctx shards one
 * longer); shard k's PreviousSig halo is the signature just before it (prev0 for the first shard), so
 * a corrupted signature at a shard edge still fails its successor in the next shard. The shards run
 * concurrently and their verdicts are merged in host memory: ok_bitmap / reject_class at their
 * positions in the whole range, first_bad = the lowest rejected ROUND over the shards (UINT64_MAX =
 * none). Identical outputs to one blsv_verify_chained call over the whole range. Replaces the serial
 * loops of client/verify.go:146-163 and chain/beacon/sync.go:100-119 on a multi-GPU node without a
 * collective (the shards share the caller's address space). Contexts are used by one thread each for
 * the duration of the call. Returns the first failing shard's code (its message in
 * blsv_last_error(ctxs[k])); BLSV_EINVAL for a bad split, a repeated context or differing groups.
 */
int blsv_verify_chained_multi(blsv_ctx* const* ctxs, size_t n_ctx, const size_t* shard_counts, uint64_t first_round,
                              const uint8_t* prev0, size_t prev0_len, const uint8_t* sigs96, size_t n,
                              uint8_t* ok_bitmap, uint64_t* first_bad, uint8_t* reject_class);

/*
 * chain.VerifyBeacon (chain/beacon.go:87-92) over n consecutive rounds first_round.. where each
 * round carries its OWN PreviousSig: prevs96[i*96 ..] (row 0 uses its first prev0_len = 32 or 96
 * bytes, every other row 96). For stored or relayed ranges whose linkage is not assumed, e.g. a
 * drand.db read by include/boltload.h (chain/boltdb/store.go:109-128 per-round Get). Outputs as in
 * blsv_verify_chained; first_bad is a ROUND.
 */
int blsv_verify_prevs(blsv_ctx* ctx, uint64_t first_round, const uint8_t* prevs96, size_t prev0_len,
                      const uint8_t* sigs96, size_t n, uint8_t* ok_bitmap, uint64_t* first_bad,
                      uint8_t* reject_class);

/*
 * One aggregator round of chain/beacon/chain.go:119-166 in two verification passes instead of three:
 * every partial verified (tbls.VerifyPartial, node.go:112; ok / reject_class per partial), Recover
 * over the first t valid shares in input order (chain.go:136; the shares it would re-verify got the
 * same deterministic verdicts in this pass), then VerifyRecovered of the group signature under the
 * group key (chain.go:141) into *group_ok. Returns BLSV_ENOTENOUGH (ok[] filled) with < t valid.
 */
int blsv_aggregate(blsv_ctx* ctx, const uint8_t* msg, size_t msg_len, const uint8_t* partials, size_t partial_len,
                   size_t k, size_t t, size_t n, uint8_t* ok, uint8_t* reject_class, uint8_t* out_sig96,
                   uint8_t* group_ok);

/* blsv_aggregate_round outcomes, in the order chain/beacon/chain.go:131-166 tests them */
#define BLSV_AGG_OK 0              /* beacon made, V1 only (fewer than t V2 partials)                   */
#define BLSV_AGG_OK_V2 1           /* beacon made with SignatureV2 (*v2_valid = VerifyRecovered V2)     */
#define BLSV_AGG_V1_RECOVER_FAIL 2 /* Recover V1 failed (< t valid distinct shares): "invalid_recovery" */
#define BLSV_AGG_V1_INVALID 3      /* VerifyRecovered V1 failed: "invalid_sig", no beacon                */
#define BLSV_AGG_V2_RECOVER_FAIL 4 /* >= t V2 partials but Recover V2 failed: no beacon (chain.go:157)  */

/*
 * The whole aggregation step of chainStore.runAggregator (chain/beacon/chain.go:131-166) for one
 * round cache, V1 and V2 together, in two verification passes: pass 1 checks the k1 V1 partials
 * (roundCache.Partials(), msg1 = chain.Message(round, prev)) and the k2 V2 partials
 * (roundCache.PartialsV2(), msg2 = chain.MessageV2(round)) in one batch (ok1/ok2); Recover V1 and,
 * when k2 >= t, Recover V2 (kyber share selection, see blsv_recover) run on the staged shares; pass 2
 * runs VerifyRecovered(pub.Commit(), ...) on both group signatures. *status = BLSV_AGG_*; sig1_96 /
 * sig2_96 hold the group signatures when produced. A V2 VerifyRecovered failure does not block the
 * beacon (*v2_valid = 0, chain.go:162-164); a V2 Recover failure does (chain.go:155-160). The
 * threshold gate (roundCache.Len() >= thr) and the cache itself stay with the caller
 * (drand_amd/callers.py Aggregator restates them).
 */
int blsv_aggregate_round(blsv_ctx* ctx, const uint8_t* msg1, size_t msg1_len, const uint8_t* partials1, size_t k1,
                         const uint8_t* msg2, size_t msg2_len, const uint8_t* partials2, size_t k2,
                         size_t partial_len, size_t t, size_t n, uint8_t* ok1, uint8_t* ok2, uint8_t* sig1_96,
                         uint8_t* sig2_96, int32_t* status, uint8_t* v2_valid);

/*
 * tbls.VerifyPartial (chain/beacon/node.go:112,125) over partials of MANY rounds in one pass:
 * partial i signs msgs[off_i .. off_i + msg_lens[i]) (messages packed back to back), e.g. a catch-up
 * of cached partials across rounds (chain/beacon/cache.go:112-182). Same outputs as
 * blsv_verify_partials. At most the context's chunk capacity of partials per call.
 */
int blsv_verify_partials_multi(blsv_ctx* ctx, const uint8_t* msgs, const uint32_t* msg_lens, const uint8_t* partials,
                               size_t partial_len, size_t k, uint8_t* ok, uint8_t* reject_class);

/*
 * chain.VerifyBeaconV2 (chain/beacon.go:94-98): msg = sha256(BE64(round)) over SignatureV2.
 * rounds may be NULL (then round i = first_round + i).
 */
int blsv_verify_unchained(blsv_ctx* ctx, const uint64_t* rounds, uint64_t first_round, const uint8_t* sigs96,
                          size_t n, uint8_t* ok_bitmap, uint64_t* first_bad, uint8_t* reject_class);

/*
 * key.Scheme.VerifyRecovered(pub, msg, sig) (chain/beacon.go:91, chain/beacon/chain.go:141,162) and
 * key.AuthScheme.Verify (key/keys.go:60-63) in batch form: message i is msgs[off_i .. off_i+len_i)
 * with msg_lens[i] bytes (consecutive), verified against pk48 (NULL = group key) and sigs96[i].
 * first_bad receives the index of the first reject.
 */
int blsv_verify_messages(blsv_ctx* ctx, const uint8_t* pk48, const uint8_t* msgs, const uint32_t* msg_lens,
                         size_t n, const uint8_t* sigs96, uint8_t* ok_bitmap, uint64_t* first_bad,
                         uint8_t* reject_class);

/*
 * key.Scheme.VerifyPartial(pubPoly, msg, partial) (chain/beacon/node.go:112,125) for k partials of
 * partial_len bytes each (98 = 2-byte BE share index || 96-byte signature); all share H(msg).
 * ok[i] = 1/0; reject_class optional.
 */
int blsv_verify_partials(blsv_ctx* ctx, const uint8_t* msg, size_t msg_len, const uint8_t* partials,
                         size_t partial_len, size_t k, uint8_t* ok, uint8_t* reject_class);

/*
 * key.Scheme.Recover(pubPoly, msg, sigs, t, n) (chain/beacon/chain.go:136,155): verifies the
 * partials and takes the first t VALID ones in input order, duplicates included (kyber tbls.Recover
 * stops at len(pubShares) >= t); those are then keyed by index as share.RecoverCommit/xyCommit does
 * (a duplicate collapses, an index >= n is dropped) and fewer than t distinct shares returns
 * BLSV_ENOTENOUGH. Otherwise Lagrange-interpolates sum lambda_i sigma_i at 0 over x = index + 1 and
 * writes the compressed 96-byte group signature. The skip-invalid / duplicate rules follow the
 * published kyber source ([ext], unpinned by any reference test).
 */
int blsv_recover(blsv_ctx* ctx, const uint8_t* msg, size_t msg_len, const uint8_t* partials, size_t partial_len,
                 size_t k, size_t t, size_t n, uint8_t* out_sig96);

/*
 * key.Scheme.Sign(priShare, msg) (chain/beacon/crypto.go:58) / AuthScheme.Sign in batch form:
 * out[i] = (index >= 0 ? BE16(index) : "") || compress(sk * H(msg_i)); sk32 is the big-endian
 * scalar (kyber Scalar.MarshalBinary), reduced mod r. Output stride 98 with index, 96 without.
 */
int blsv_sign(blsv_ctx* ctx, const uint8_t* sk32, int32_t index, const uint8_t* msgs, const uint32_t* msg_lens,
              size_t n, uint8_t* out);

/* ---------------------------------------------------------------- device-resident batches */

/*
 * Chained verify over HBM-resident signatures, optionally split into independently seeded
 * segments of seg_len rounds (seg_len = 0 means one segment): with s = (i + seg_phase) / seg_len,
 * beacon i (round first_round + i) uses d_seeds96[s] as PreviousSig when i == 0 or
 * (i + seg_phase) % seg_len == 0 (length seed0_len for s = 0, else 96), else d_sigs96[i-1].
 * seg_phase (< seg_len; 0 when segments start at item 0) lets a shard that begins inside a
 * segment pass its one-signature halo as d_seeds96[0] (multi-GPU range sharding).
 * Outputs (device): d_bitmap (ceil(n/64) uint64 words, fully written), d_first_bad (one uint64:
 * the ROUND of the first reject or UINT64_MAX), d_reject_class (optional, n bytes). Asynchronous
 * on `stream` (a hipStream_t; NULL = the context stream). The context's staging buffers are shared
 * by every call: successive *_dev calls on one context must be issued on ONE stream (or the caller
 * orders them with events), never concurrently on two streams. Internally the decompression stage
 * runs on the context's side stream, forked from `stream` after the work already queued there and
 * joined back into it (events) before the pairing stage: ordering with respect to `stream` holds.
 */
int blsv_verify_chained_dev(blsv_ctx* ctx, uint64_t first_round, uint64_t seg_len, uint64_t seg_phase,
                            const uint8_t* d_seeds96, size_t seed0_len, const uint8_t* d_sigs96, size_t n,
                            uint64_t* d_bitmap, uint64_t* d_first_bad, uint8_t* d_reject_class, void* stream);

/*
 * Synthetic chained history (client/test/result/mock/result.go:98-132, per segment, on device):
 * d_sigs96[i] = compress(sk * H(Message(first_round + i, prev))) with the seed rule above
 * (seg_phase = 0). Same single-stream rule as blsv_verify_chained_dev.
 */
int blsv_generate_chained_dev(blsv_ctx* ctx, const uint8_t* sk32, uint64_t first_round, uint64_t seg_len,
                              const uint8_t* d_seeds96, size_t seed0_len, uint8_t* d_sigs96, size_t n, void* stream);

/* Wait for the context stream. */
int blsv_synchronize(blsv_ctx* ctx);

/*
 * Latency-path cutover (see the latency contract above): calls with 1..lat_max items take the latency
 * path, larger ones the batch pipeline; 0 = batch pipeline only. The default is the BLSV_LAT_MAX
 * environment variable (a non-negative decimal integer; anything else is ignored with a warning on
 * stderr), else 1536 (below where the two paths cross on MI355X, ~1,750 items). Values above 2^20 (one pipeline chunk)
 * are clamped to 2^20. Returns the previous value.
 */
size_t blsv_set_lat_max(blsv_ctx* ctx, size_t lat_max);

/*
 * Memory contract. A context allocates its pipeline staging lazily, for min(largest batch, chunk)
 * items at ~42.4 KB per item (39 KB of it the Miller line staging): a lone verify or a round of
 * partials takes a few MB, a full 2^20 chunk ~43 GB of the GPU's 288 GB. The chunk defaults to 2^20
 * (the BLSV_CHUNK environment variable overrides it); a larger batch runs in chunk-sized passes with
 * identical verdicts. When an allocation fails with out-of-memory the context frees its staging,
 * halves its chunk (not below 16,384 items) and retries, so contexts or ranks sharing one GPU degrade
 * to smaller passes instead of failing. blsv_set_chunk caps it explicitly (items, rounded up to a
 * multiple of 64 and clamped to [16384, 2^20]; 0 = the default) and releases the staging at once when
 * it shrinks; it also clamps lat_max. Returns the previous chunk.
 */
size_t blsv_set_chunk(blsv_ctx* ctx, size_t items);
/* HBM bytes of pipeline staging the context holds now (0 before its first batch). */
size_t blsv_workspace_bytes(const blsv_ctx* ctx);

/* ---------------------------------------------------------------- thread-safe service
 *
 * Concurrent single-item callers: the reference verifies each arrival in its own goroutine -- one per
 * partial packet (core/drand_public.go:39 -> chain/beacon/node.go:112,125), one per gossip message
 * (lp2p/client/validator.go:64), one per client.Get (client/verify.go:185-207). A blsv_service may be
 * called from any number of threads at once. Each call blocks until its item is verified; the items of
 * calls that arrive close together are coalesced into ONE launch (the latency path up to lat_max
 * items, the batch pipeline beyond) by the service's dispatcher thread, and every caller gets its own
 * verdict. Coalescing window: after the first waiting item the dispatcher keeps gathering while new
 * items keep arriving within gap_us of the previous one, for at most max_wait_us (0, 0 = the defaults
 * 100 us and 2000 us; the BLSV_SVC_GAP_US / BLSV_SVC_MAX_WAIT_US environment variables override the
 * defaults); items that arrive while a launch runs form the next batch. The service owns one context
 * whose chunk is capped at 65,536 items (~2.7 GB of staging at most).
 */
typedef struct blsv_service blsv_service;

int blsv_service_create(int device, uint32_t gap_us, uint32_t max_wait_us, blsv_service** out);
/* Waits for the items already submitted, then stops the dispatcher. No call may be in flight or follow. */
void blsv_service_destroy(blsv_service* svc);

/*
 * key.Scheme.VerifyPartial(pubPoly, msg, partial) (chain/beacon/node.go:112,125): the group is passed
 * with every call as its t commitments (48 bytes each) and size n, like the reference's per-call
 * *share.PubPoly; the service keeps the PK_i tables of the groups it has seen (reshare transitions keep
 * two alive). *ok = 1/0, *reject_class (optional) = BLSV_REJ_*. Returns BLSV_EINVAL for a group whose
 * commitments do not decode (the call's own error, other callers are unaffected).
 */
int blsv_service_verify_partial(blsv_service* svc, const uint8_t* commits48, size_t t, size_t n, const uint8_t* msg,
                                size_t msg_len, const uint8_t* partial, size_t partial_len, uint8_t* ok,
                                uint8_t* reject_class);

/*
 * key.Scheme.VerifyRecovered(pub, msg, sig) (chain/beacon.go:91 via chain.VerifyBeacon; the gossip
 * validator and client.Get verify one beacon each) against the 48-byte compressed G1 key pk48.
 * Returns BLSV_EINVAL for a key that does not decode (kilic G1.FromCompressed).
 */
int blsv_service_verify_recovered(blsv_service* svc, const uint8_t* pk48, const uint8_t* msg, size_t msg_len,
                                  const uint8_t* sig96, uint8_t* ok, uint8_t* reject_class);

/* Counters since creation: launches, items verified, the largest batch. Any pointer may be NULL. */
int blsv_service_stats(blsv_service* svc, uint64_t* launches, uint64_t* items, uint64_t* max_batch);

#ifdef __cplusplus
}
#endif

#endif /* DRAND_AMD_BLSVERIFY_H */
