/*
 * Bulk loader of drand's beacon store (drand.db, go.etcd.io/bbolt v1.3.4) into the SoA layout that
 * blsv_verify_chained takes. SURVEY.md §8f rank 2. Host-only (no device code).
 *
 * Replaces the per-round reads of chain/boltdb/store.go:109-128 (boltStore.Get) and the cursor
 * walk of store.go:137-160 (Cursor) when a node's whole history is verified offline: one mmap,
 * one B+tree walk of bucket "beacons" (store.go:21), hexjson values (chain/beacon.go:35-43)
 * decoded straight into round / prev / signature arrays.
 *
 * Return codes: 0 = success, -1 = error (text from dl_last_error; the handle stays valid for it
 * even when dl_open fails, and must be passed to dl_close).
 */
#ifndef DRAND_AMD_BOLTLOAD_H
#define DRAND_AMD_BOLTLOAD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct dl_db dl_db;

/* Open (read-only mmap) and index bucket "beacons" in key (= round) order. */
int dl_open(const char* path, dl_db** out);

/* Number of entries in bucket "beacons" (boltStore.Len, store.go:47-58). */
int64_t dl_count(const dl_db* db);

/*
 * Decode entries [start, start + max_n) into caller-owned arrays of n = min(max_n, count - start):
 * rounds[n]; prev96[n*96] + prev_len[n]; sigs96[n*96] + sig_len[n]; optional sigs_v2_96[n*96] +
 * v2_len[n] (may be NULL). Byte fields are zero-padded to 96; a length above 96 is reported as 255.
 * Fails if a value is not a beacon object or its Round differs from the 8-byte big-endian key.
 */
int dl_load(dl_db* db, size_t start, size_t max_n, uint64_t* rounds, uint8_t* prev96, uint8_t* prev_len,
            uint8_t* sigs96, uint8_t* sig_len, uint8_t* sigs_v2_96, uint8_t* v2_len, size_t* n_out);

const char* dl_last_error(const dl_db* db);
void dl_close(dl_db* db);

#ifdef __cplusplus
}
#endif
#endif
