/*
 * cabi_smoke -- the C ABI of libblsverify.so exercised from a plain C process: no Python, no torch,
 * only the library and /opt/rocm's HIP runtime, i.e. exactly what a cgo caller (gpu/blsverify,
 * INTEGRATION.md) loads. Checks against the committed fixture tests/golden/cabi_vectors.txt
 * (derived from tests/golden/golden.json by tests/golden/make_cabi_vectors.py):
 *
 *   1. chain.VerifyBeacon over the 24-round golden chain (blsv_verify_chained): all accept;
 *   2. one corrupted signature: exactly rounds i and i+1 reject, first_bad = round i;
 *   3. the reference KAT key/curve_test.go:10-30: blsv_sign reproduces the 96-byte signature and
 *      blsv_verify_messages accepts it (and rejects it under another message);
 *   4. the golden n=64/t=33 threshold round: every partial verifies, Recover of a shuffled
 *      33-subset is the group signature, blsv_aggregate_round gives the V1 and V2 group signatures;
 *   5. latency of one lone VerifyRecovered (blsv_verify_messages, n = 1);
 *   6. the thread-safe service (blsv_service_*): 64 pthreads each verify ONE golden partial at the
 *      same moment (one corrupted), every verdict right, the wall time of all 64 against a lone call.
 *
 * Prints one line per check and "cabi_smoke ok" at the end; exit status 0 only if all pass.
 * Build: make -C tools cabi_smoke (gcc, links -lblsverify with an rpath to drand_amd/).
 */
#define _POSIX_C_SOURCE 200112L
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>
#include <time.h>

#include "../include/blsverify.h"

#define MAXV 256

typedef struct {
  char key[32];
  uint8_t* data;
  size_t len;
} vec_t;

static vec_t V[MAXV];
static int nv = 0;
static int failures = 0;

static int hexval(int c) {
  if (c >= '0' && c <= '9') return c - '0';
  if (c >= 'a' && c <= 'f') return c - 'a' + 10;
  if (c >= 'A' && c <= 'F') return c - 'A' + 10;
  return -1;
}

static int load(const char* path) {
  FILE* f = fopen(path, "r");
  if (!f) {
    perror(path);
    return -1;
  }
  static char line[1 << 16];
  while (fgets(line, sizeof line, f) && nv < MAXV) {
    char* sp = strchr(line, ' ');
    if (!sp || line[0] == '#') continue;
    *sp = 0;
    char* hx = sp + 1;
    size_t n = strcspn(hx, "\r\n");
    vec_t* v = &V[nv++];
    snprintf(v->key, sizeof v->key, "%.31s", line);
    v->len = n / 2;
    v->data = (uint8_t*)malloc(v->len + 1);
    for (size_t i = 0; i < v->len; i++) v->data[i] = (uint8_t)(hexval(hx[2 * i]) << 4 | hexval(hx[2 * i + 1]));
  }
  fclose(f);
  return 0;
}

/* k-th vector named key (0-based among equal keys) */
static const vec_t* get(const char* key, int k) {
  for (int i = 0; i < nv; i++)
    if (strcmp(V[i].key, key) == 0 && k-- == 0) return &V[i];
  fprintf(stderr, "missing vector %s\n", key);
  exit(2);
}

static int count(const char* key) {
  int c = 0;
  for (int i = 0; i < nv; i++) c += strcmp(V[i].key, key) == 0;
  return c;
}

static void check(int cond, const char* what) {
  printf("%s %s\n", cond ? "PASS" : "FAIL", what);
  if (!cond) failures++;
}

/* 6. one thread of the service burst: waits at the barrier, verifies its partial */
typedef struct {
  blsv_service* svc;
  const uint8_t *commits, *msg, *partial;
  size_t t, n, msg_len;
  pthread_barrier_t* bar;
  uint8_t ok, cls;
  int rc;
} svc_job_t;

static void* svc_worker(void* p) {
  svc_job_t* j = (svc_job_t*)p;
  pthread_barrier_wait(j->bar);
  j->rc = blsv_service_verify_partial(j->svc, j->commits, j->t, j->n, j->msg, j->msg_len, j->partial, 98, &j->ok,
                                      &j->cls);
  return NULL;
}

static double now_ms(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec * 1e3 + ts.tv_nsec / 1e6;
}

#define RC(expr)                                                                     \
  do {                                                                               \
    int rc_ = (expr);                                                                \
    if (rc_ != BLSV_OK) {                                                            \
      fprintf(stderr, "%s -> %d: %s\n", #expr, rc_, blsv_last_error(ctx));           \
      return 1;                                                                      \
    }                                                                                \
  } while (0)

int main(int argc, char** argv) {
  const char* path = argc > 1 ? argv[1] : "tests/golden/cabi_vectors.txt";
  if (load(path)) return 2;
  blsv_ctx* ctx = NULL;
  double t0 = now_ms();
  if (blsv_create(0, &ctx) != BLSV_OK) {
    fprintf(stderr, "blsv_create failed (no HIP device?)\n");
    return 1;
  }
  printf("INFO %s, context up in %.1f ms\n", blsv_version(), now_ms() - t0);

  /* 1. golden chain */
  const int n = count("sig");
  uint8_t* sigs = (uint8_t*)malloc((size_t)n * 96);
  for (int i = 0; i < n; i++) memcpy(sigs + 96 * i, get("sig", i)->data, 96);
  const vec_t* pk = get("pk", 0);
  const vec_t* seed = get("seed", 0);
  RC(blsv_set_group(ctx, pk->data, 1, 1));
  uint8_t bm[64] = {0}, cls[256] = {0};
  uint64_t fb = 0;
  RC(blsv_verify_chained(ctx, 1, seed->data, seed->len, sigs, (size_t)n, bm, &fb, cls));
  int all = 1;
  for (int i = 0; i < n; i++) all &= (bm[i / 8] >> (i % 8)) & 1;
  check(all && fb == UINT64_MAX, "verify_chained: 24 golden rounds accept");

  /* 2. corrupted signature 3 (round 4): rounds 4 and 5 reject */
  sigs[3 * 96 + 50] ^= 1;
  RC(blsv_verify_chained(ctx, 1, seed->data, seed->len, sigs, (size_t)n, bm, &fb, cls));
  int exact = 1;
  for (int i = 0; i < n; i++) exact &= (((bm[i / 8] >> (i % 8)) & 1) == (i != 3 && i != 4));
  check(exact && fb == 4, "verify_chained: corrupted round 4 -> rounds 4, 5 reject, first_bad = 4");
  sigs[3 * 96 + 50] ^= 1;

  /* 3. KAT key/curve_test.go:10-30 */
  const vec_t *ksk = get("kat_sk", 0), *kmsg = get("kat_msg", 0), *ksig = get("kat_sig", 0), *kpk = get("kat_pk", 0);
  uint8_t out[98];
  uint32_t klen = (uint32_t)kmsg->len;
  RC(blsv_sign(ctx, ksk->data, -1, kmsg->data, &klen, 1, out));
  check(memcmp(out, ksig->data, 96) == 0, "sign: KAT signature byte-exact");
  uint8_t one = 0, c1 = 0;
  RC(blsv_verify_messages(ctx, kpk->data, kmsg->data, &klen, 1, ksig->data, &one, &fb, &c1));
  check((one & 1) && fb == UINT64_MAX, "verify_messages: KAT accepts");
  uint32_t mlen = 32;
  RC(blsv_verify_messages(ctx, kpk->data, seed->data, &mlen, 1, ksig->data, &one, &fb, &c1));
  check(!(one & 1) && c1 == BLSV_REJ_PAIRING && fb == 0, "verify_messages: KAT signature under another message rejects");

  /* 4. threshold round */
  const int t = (int)get("t", 0)->data[0], gn = (int)get("n", 0)->data[0];
  const int nc = count("commit");
  uint8_t* commits = (uint8_t*)malloc((size_t)nc * 48);
  for (int i = 0; i < nc; i++) memcpy(commits + 48 * i, get("commit", i)->data, 48);
  RC(blsv_set_group(ctx, commits, (size_t)nc, (size_t)gn));
  const vec_t *msg1 = get("msg", 0), *msg2 = get("msg_v2", 0);
  const int np = count("partial");
  uint8_t *p1 = (uint8_t*)malloc((size_t)np * 98), *p2 = (uint8_t*)malloc((size_t)np * 98);
  for (int i = 0; i < np; i++) {
    memcpy(p1 + 98 * i, get("partial", i)->data, 98);
    memcpy(p2 + 98 * i, get("partial_v2", i)->data, 98);
  }
  uint8_t okv[128], okv2[128], rcls[128];
  RC(blsv_verify_partials(ctx, msg1->data, msg1->len, p1, 98, (size_t)np, okv, rcls));
  int allp = 1;
  for (int i = 0; i < np; i++) allp &= okv[i];
  check(allp, "verify_partials: 64 golden partials accept");
  const int ns = count("subset");
  uint8_t* sub = (uint8_t*)malloc((size_t)ns * 98);
  for (int i = 0; i < ns; i++) memcpy(sub + 98 * i, get("subset", i)->data, 98);
  uint8_t gsig[96], gsig2[96];
  RC(blsv_recover(ctx, msg1->data, msg1->len, sub, 98, (size_t)ns, (size_t)t, (size_t)gn, gsig));
  check(memcmp(gsig, get("group_sig", 0)->data, 96) == 0, "recover: shuffled 33-subset -> group signature byte-exact");
  int32_t status = -1;
  uint8_t v2ok = 0;
  double ta = now_ms();
  RC(blsv_aggregate_round(ctx, msg1->data, msg1->len, p1, (size_t)np, msg2->data, msg2->len, p2, (size_t)np, 98,
                          (size_t)t, (size_t)gn, okv, okv2, gsig, gsig2, &status, &v2ok));
  double agg_ms = now_ms() - ta;
  check(status == BLSV_AGG_OK_V2 && v2ok && memcmp(gsig, get("group_sig", 0)->data, 96) == 0 &&
            memcmp(gsig2, get("group_sig_v2", 0)->data, 96) == 0,
        "aggregate_round: V1 + V2 group signatures byte-exact");
  printf("INFO aggregate_round n=%d t=%d (V1+V2, %d partials): %.1f ms (first call)\n", gn, t, 2 * np, agg_ms);
  /* warm: the fused V1 round (VerifyPartial x n + Recover + VerifyRecovered) and the V1+V2 round */
  double best_agg = 1e30, best_round = 1e30;
  for (int r = 0; r < 5; r++) {
    uint8_t gok = 0;
    double a = now_ms();
    RC(blsv_aggregate(ctx, msg1->data, msg1->len, p1, 98, (size_t)np, (size_t)t, (size_t)gn, okv, rcls, gsig, &gok));
    double d = now_ms() - a;
    best_agg = d < best_agg ? d : best_agg;
    check(gok && memcmp(gsig, get("group_sig", 0)->data, 96) == 0, "aggregate (warm): group signature byte-exact");
    a = now_ms();
    RC(blsv_aggregate_round(ctx, msg1->data, msg1->len, p1, (size_t)np, msg2->data, msg2->len, p2, (size_t)np, 98,
                            (size_t)t, (size_t)gn, okv, okv2, gsig, gsig2, &status, &v2ok));
    d = now_ms() - a;
    best_round = d < best_round ? d : best_round;
  }
  printf("INFO warm fused round n=%d t=%d (blsv_aggregate, %d partials): %.2f ms\n", gn, t, np, best_agg);
  printf("INFO warm aggregate_round V1+V2 (%d partials): %.2f ms\n", 2 * np, best_round);

  /* 5. lone VerifyRecovered latency (warm, best of 5) */
  RC(blsv_set_group(ctx, pk->data, 1, 1));
  double best = 1e30;
  for (int r = 0; r < 5; r++) {
    double a = now_ms();
    RC(blsv_verify_chained(ctx, 1, seed->data, seed->len, sigs, 1, bm, &fb, cls));
    double d = now_ms() - a;
    best = d < best ? d : best;
  }
  check(bm[0] & 1, "verify_chained: lone round 1 accepts");
  printf("INFO lone verify latency: %.2f ms\n", best);

  /* 6. the Go host's multi-GPU shape: one context per GPU (device k % count), the continuous 2,049-round
   * chain split 3 ways at unaligned edges, a corrupted signature at a shard's end whose successor (the
   * next shard's first round) must reject through the halo; merged = one whole-history call */
  {
    const char* cpath = argc > 2 ? argv[2] : "tests/golden/chain2049.bin";
    FILE* cf = fopen(cpath, "rb");
    enum { CN = 2049, NC = 3 };
    uint8_t* chain = (uint8_t*)malloc((size_t)CN * 96);
    const size_t got = cf ? fread(chain, 96, CN, cf) : 0;
    if (cf) fclose(cf);
    check(got == CN, "multi: chain2049.bin read");
    if (got == CN) {
      const int ndev = blsv_device_count();
      blsv_ctx* cs[NC] = {NULL, NULL, NULL};
      int up = ndev > 0;
      for (int k = 0; k < NC && up; k++) up = blsv_create(k % ndev, &cs[k]) == BLSV_OK &&
                                              blsv_set_group(cs[k], pk->data, 1, 1) == BLSV_OK;
      check(up, "multi: three contexts with the chain key");
      const size_t counts[NC] = {700, 1, 1348};
      const int hit[3] = {699, 700, 1500}; /* shard 0's last, shard 1's only, mid shard 2 */
      for (int h = 0; h < 3; h++) chain[hit[h] * 96 + 50] ^= 4;
      static uint8_t wbm[(CN + 7) / 8], mbm[(CN + 7) / 8], wcls[CN], mcls[CN];
      uint64_t wfb = 0, mfb = 0;
      if (up) {
        RC(blsv_set_group(ctx, pk->data, 1, 1));
        RC(blsv_verify_chained(ctx, 1, seed->data, seed->len, chain, CN, wbm, &wfb, wcls));
        double a = now_ms();
        int rc = blsv_verify_chained_multi(cs, NC, counts, 1, seed->data, seed->len, chain, CN, mbm, &mfb, mcls);
        double d = now_ms() - a;
        int exact = rc == BLSV_OK && memcmp(wbm, mbm, sizeof wbm) == 0 && memcmp(wcls, mcls, CN) == 0 && wfb == mfb &&
                    mfb == 700;
        for (int i = 0; i < CN; i++) {
          const int bad = i == 699 || i == 700 || i == 701 || i == 1500 || i == 1501;
          exact &= ((mbm[i / 8] >> (i % 8)) & 1) == !bad;
        }
        check(exact, "multi: 3 contexts over a 700/1/1348 split = the whole-history call (halo-linked rejects)");
        printf("INFO verify_chained_multi: %d contexts on %d device(s), %d rounds in %.2f ms\n", NC, ndev, CN, d);
      }
      for (int k = 0; k < NC; k++) blsv_destroy(cs[k]);
    }
    free(chain);
  }

  /* 7. the service under 64 concurrent callers */
  {
    blsv_service* svc = NULL;
    RC(blsv_service_create(0, 0, 0, &svc));
    /* the corrupted share and its exact reject class, both from the oracle-made vector file */
    uint8_t bad[98];
    memcpy(bad, get("bad_partial", 0)->data, 98);
    const uint8_t bad_cls = get("bad_partial_class", 0)->data[0];
    uint8_t o = 0, k = 0;
    RC(blsv_service_verify_partial(svc, commits, (size_t)nc, (size_t)gn, msg1->data, msg1->len, p1, 98, &o, &k));
    check(o == 1 && k == 0, "service: lone partial accepts (warm-up)");
    double lone = 1e30;
    for (int r = 0; r < 5; r++) {
      double a = now_ms();
      RC(blsv_service_verify_partial(svc, commits, (size_t)nc, (size_t)gn, msg1->data, msg1->len, p1 + 98, 98, &o,
                                     &k));
      double d = now_ms() - a;
      lone = d < lone ? d : lone;
    }
    enum { NT = 64 };
    svc_job_t jobs[NT];
    pthread_t th[NT];
    pthread_barrier_t bar;
    double burst = 1e30;
    int right = 1;
    for (int rep = 0; rep < 3; rep++) {
      pthread_barrier_init(&bar, NULL, NT + 1);
      for (int i = 0; i < NT; i++) {
        jobs[i] = (svc_job_t){svc, commits, msg1->data, i == 5 ? bad : p1 + 98 * (i % np), (size_t)nc, (size_t)gn,
                              msg1->len, &bar, 0, 0, 0};
        pthread_create(&th[i], NULL, svc_worker, &jobs[i]);
      }
      pthread_barrier_wait(&bar);
      double a = now_ms();
      for (int i = 0; i < NT; i++) pthread_join(th[i], NULL);
      double d = now_ms() - a;
      burst = d < burst ? d : burst;
      pthread_barrier_destroy(&bar);
      for (int i = 0; i < NT; i++)
        right &= jobs[i].rc == 0 && jobs[i].ok == (i != 5) && jobs[i].cls == (i == 5 ? bad_cls : 0);
    }
    uint64_t la = 0, it = 0, mb = 0;
    RC(blsv_service_stats(svc, &la, &it, &mb));
    check(right, "service: 64 concurrent VerifyPartial, each verdict and class = the oracle's");
    /* measured 1.3-1.5x over round 5 (profiles/r05*_cabi_smoke.txt); an uncoalesced service is ~64x */
    check(burst <= 3.0 * lone, "service: 64 concurrent calls within 3x one lone call");
    printf("INFO service: lone VerifyPartial %.2f ms, 64 concurrent %.2f ms (best of 3), %llu launches for %llu items,"
           " largest batch %llu\n",
           lone, burst, (unsigned long long)la, (unsigned long long)it, (unsigned long long)mb);
    blsv_service_destroy(svc);
  }

  blsv_destroy(ctx);
  printf("%s (%d failures)\n", failures ? "cabi_smoke FAILED" : "cabi_smoke ok", failures);
  return failures ? 1 : 0;
}
