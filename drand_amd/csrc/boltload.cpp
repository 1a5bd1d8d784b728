// Bulk loader of a drand node's beacon store (drand.db, bbolt) into the engine's SoA batch layout.
// SURVEY.md §8f rank 2. Host-only code (no HIP): it feeds blsv_verify_chained.
//
// What drand writes (chain/boltdb/store.go:21,68-81): bucket "beacons", key = 8-byte big-endian
// round (chain.RoundToBytes, chain/store.go:227-231), value = hexjson chain.Beacon
// (chain/beacon.go:35-43: {"PreviousSig":"<hex>","Round":N,"Signature":"<hex>"[,"SignatureV2":"<hex>"]}).
//
// The file format is go.etcd.io/bbolt v1.3.4 (go.mod:37), not vendored here. Restated from its
// published layout: pages of meta.pageSize bytes; a 16-byte page header {id u64, flags u16,
// count u16, overflow u32}; two meta pages (0 and 1) {magic 0xED0CDAED, version 2, pageSize, flags,
// root bucket {root pgid, sequence}, freelist pgid, high-water pgid, txid, checksum = FNV-1a-64 of
// the 56 bytes before it}, the valid one with the larger txid wins; branch elements {pos u32,
// ksize u32, pgid u64}, leaf elements {flags u32, pos u32, ksize u32, vsize u32} with pos relative to
// the element; a sub-bucket is a leaf value with flag 0x01 holding {root pgid, sequence} and, when
// root == 0, an inline page right after it. Parity against files written by bbolt itself is
// unpinned: the reference holds no drand.db fixture.
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <thread>
#include <cstdio>
#include <cctype>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/boltload.h"

namespace {

constexpr uint32_t kMagic = 0xED0CDAEDu;
constexpr uint16_t kBranch = 0x01, kLeaf = 0x02, kMeta = 0x04;
constexpr uint32_t kBucketLeaf = 0x01;
constexpr size_t kPageHdr = 16;

template <class T> T rd(const uint8_t* p) { T v; std::memcpy(&v, p, sizeof v); return v; }  // little-endian host

struct Entry {
    const uint8_t* k; uint32_t ks;
    const uint8_t* v; uint32_t vs;
};

}  // namespace

struct dl_db {
    int fd = -1;
    const uint8_t* base = nullptr;
    size_t size = 0;
    uint32_t page_size = 0;
    uint64_t bucket_root = 0;            // 0 = inline bucket
    const uint8_t* inline_page = nullptr;
    const uint8_t* inline_end = nullptr;  // end of the bucket value holding the inline page
    std::vector<Entry> entries;          // "beacons" in key order
    std::string err;
};

namespace {

int fail(dl_db* db, const std::string& m) { db->err = m; return -1; }

uint64_t fnv64a(const uint8_t* p, size_t n) {
    uint64_t h = 0xcbf29ce484222325ull;
    for (size_t i = 0; i < n; i++) { h ^= p[i]; h *= 0x100000001b3ull; }
    return h;
}

const uint8_t* page_at(dl_db* db, uint64_t id) {
    if (db->page_size == 0 || id > (db->size / db->page_size)) return nullptr;
    uint64_t off = id * db->page_size;
    if (off + kPageHdr > db->size) return nullptr;
    return db->base + off;
}

// In-order walk of a B+tree rooted at page `p` (which may be an inline page: `limit` bounds it).
int walk(dl_db* db, const uint8_t* p, const uint8_t* limit, std::vector<Entry>& out, int depth) {
    if (depth > 64) return fail(db, "tree too deep (corrupt file)");
    if (p + kPageHdr > limit) return fail(db, "page header out of range");
    uint16_t flags = rd<uint16_t>(p + 8), count = rd<uint16_t>(p + 10);
    uint32_t overflow = rd<uint32_t>(p + 12);
    const uint8_t* end = limit;
    if (limit == db->base + db->size) {
        uint64_t span = uint64_t(db->page_size) * (uint64_t(overflow) + 1);
        if (p + span <= limit) end = p + span;
    }
    const uint8_t* el = p + kPageHdr;
    if (el + size_t(count) * 16 > end) return fail(db, "element table out of range");
    if (flags & kBranch) {
        for (uint16_t i = 0; i < count; i++) {
            uint64_t child = rd<uint64_t>(el + 16 * i + 8);
            const uint8_t* c = page_at(db, child);
            if (!c) return fail(db, "branch child out of range");
            if (walk(db, c, db->base + db->size, out, depth + 1)) return -1;
        }
        return 0;
    }
    if (!(flags & kLeaf)) return fail(db, "unexpected page type");
    for (uint16_t i = 0; i < count; i++) {
        const uint8_t* e = el + 16 * i;
        uint32_t f = rd<uint32_t>(e), pos = rd<uint32_t>(e + 4), ks = rd<uint32_t>(e + 8), vs = rd<uint32_t>(e + 12);
        const uint8_t* k = e + pos;
        if (k < db->base || k + uint64_t(ks) + vs > end) return fail(db, "leaf element out of range");
        if (f & kBucketLeaf) continue;   // nested buckets are not part of drand's layout
        out.push_back({k, ks, k + ks, vs});
    }
    return 0;
}

// Find bucket `name` among the root bucket's entries (leaf values flagged as buckets).
int find_bucket(dl_db* db, const uint8_t* p, const char* name, int depth) {
    if (depth > 64) return fail(db, "tree too deep (corrupt file)");
    uint16_t flags = rd<uint16_t>(p + 8), count = rd<uint16_t>(p + 10);
    const uint8_t* el = p + kPageHdr;
    if (el + size_t(count) * 16 > db->base + db->size) return fail(db, "root element table out of range");
    size_t nl = std::strlen(name);
    for (uint16_t i = 0; i < count; i++) {
        const uint8_t* e = el + 16 * i;
        if (flags & kBranch) {
            const uint8_t* c = page_at(db, rd<uint64_t>(e + 8));
            if (!c) return fail(db, "root branch child out of range");
            int r = find_bucket(db, c, name, depth + 1);
            if (r <= 0) return r;
            continue;
        }
        uint32_t f = rd<uint32_t>(e), pos = rd<uint32_t>(e + 4), ks = rd<uint32_t>(e + 8), vs = rd<uint32_t>(e + 12);
        const uint8_t* k = e + pos;
        if (k + uint64_t(ks) + vs > db->base + db->size) return fail(db, "root leaf element out of range");
        if ((f & kBucketLeaf) && ks == nl && std::memcmp(k, name, nl) == 0) {
            if (vs < 16) return fail(db, "bucket header truncated");
            db->bucket_root = rd<uint64_t>(k + ks);
            if (db->bucket_root == 0) {
                if (vs < 16 + kPageHdr) return fail(db, "inline bucket truncated");
                db->inline_page = k + ks + 16;
                db->inline_end = k + ks + vs;
            }
            return 0;
        }
    }
    return 1;  // not here
}

struct HexLut {
    int8_t v[256];
    HexLut() {
        for (int c = 0; c < 256; c++) v[c] = -1;
        for (int c = '0'; c <= '9'; c++) v[c] = int8_t(c - '0');
        for (int c = 'a'; c <= 'f'; c++) v[c] = int8_t(c - 'a' + 10);
        for (int c = 'A'; c <= 'F'; c++) v[c] = int8_t(c - 'A' + 10);
    }
};
const HexLut kHex;

inline int hexval(uint8_t c) { return kHex.v[c]; }

// Decode a hex string value into out (cap bytes); returns byte length, or -1 on malformed hex.
long hexdecode(const uint8_t* s, size_t n, uint8_t* out, size_t cap) {
    if (n % 2) return -1;
    size_t m = n / 2;
    for (size_t i = 0; i < m; i++) {
        int a = hexval(s[2 * i]), b = hexval(s[2 * i + 1]);
        if (a < 0 || b < 0) return -1;
        if (i < cap) out[i] = uint8_t(a << 4 | b);
    }
    return long(m);
}

const uint8_t* skip_ws(const uint8_t* p, const uint8_t* e) {
    while (p < e && (*p == ' ' || *p == '\n' || *p == '\r' || *p == '\t')) p++;
    return p;
}

struct Fields {
    uint64_t round = 0;
    long prev_len = 0, sig_len = 0, v2_len = 0;
};

// Minimal parser for the flat object hexjson writes for chain.Beacon: string keys, string (hex) or
// unsigned-integer values, no nesting, no escapes inside the values it reads.
int parse_beacon(const uint8_t* p, size_t n, Fields& f, uint8_t* prev, uint8_t* sig, uint8_t* v2) {
    const uint8_t* e = p + n;
    p = skip_ws(p, e);
    if (p >= e || *p != '{') return -1;
    p++;
    for (;;) {
        p = skip_ws(p, e);
        if (p < e && *p == '}') return 0;
        if (p >= e || *p != '"') return -1;
        const uint8_t* ks = ++p;
        while (p < e && *p != '"') p++;
        if (p >= e) return -1;
        // encoding/json (which hexjson forks) matches field names case-insensitively
        std::string key(reinterpret_cast<const char*>(ks), size_t(p - ks));
        for (auto& ch : key) ch = char(std::tolower((unsigned char)ch));
        p = skip_ws(p + 1, e);
        if (p >= e || *p != ':') return -1;
        p = skip_ws(p + 1, e);
        if (p >= e) return -1;
        if (*p == '"') {
            const uint8_t* vs = ++p;
            while (p < e && *p != '"') p++;
            if (p >= e) return -1;
            size_t vn = size_t(p - vs);
            p++;
            long len = 0;
            if (key == "previoussig") len = f.prev_len = hexdecode(vs, vn, prev, 96);
            else if (key == "signature") len = f.sig_len = hexdecode(vs, vn, sig, 96);
            else if (key == "signaturev2") len = f.v2_len = hexdecode(vs, vn, v2, 96);
            if (len < 0) return -1;
        } else if (*p >= '0' && *p <= '9') {
            uint64_t v = 0;
            while (p < e && *p >= '0' && *p <= '9') {
                const uint64_t d = uint64_t(*p++ - '0');
                if (v > (UINT64_MAX - d) / 10) return -1;  // json.Unmarshal: overflows uint64
                v = v * 10 + d;
            }
            if (key == "round") f.round = v;
        } else if (e - p >= 4 && std::memcmp(p, "null", 4) == 0) {
            p += 4;
        } else {
            return -1;
        }
        p = skip_ws(p, e);
        if (p < e && *p == ',') { p++; continue; }
        if (p < e && *p == '}') return 0;
        return -1;
    }
}

}  // namespace

extern "C" {

int dl_open(const char* path, dl_db** out) {
    if (!path || !out) return -1;
    *out = nullptr;
    dl_db* db = new dl_db();
    *out = db;
    db->fd = ::open(path, O_RDONLY);
    if (db->fd < 0) return fail(db, std::string("cannot open ") + path);
    struct stat st;
    if (fstat(db->fd, &st) != 0 || st.st_size < 1024) return fail(db, "file too small for a bbolt database");
    db->size = size_t(st.st_size);
    void* m = mmap(nullptr, db->size, PROT_READ, MAP_PRIVATE, db->fd, 0);
    if (m == MAP_FAILED) return fail(db, "mmap failed");
    db->base = static_cast<const uint8_t*>(m);

    // meta page 0 tells the page size; meta page 1 sits at page_size.
    const uint8_t* best = nullptr;
    uint64_t best_tx = 0;
    uint32_t ps0 = rd<uint32_t>(db->base + kPageHdr + 8);
    for (int i = 0; i < 2; i++) {
        size_t off = i == 0 ? 0 : ps0;
        if (ps0 < 512 || off + kPageHdr + 64 > db->size) continue;
        const uint8_t* pg = db->base + off;
        const uint8_t* m8 = pg + kPageHdr;
        if (!(rd<uint16_t>(pg + 8) & kMeta)) continue;
        if (rd<uint32_t>(m8) != kMagic || rd<uint32_t>(m8 + 4) != 2) continue;
        if (fnv64a(m8, 56) != rd<uint64_t>(m8 + 56)) continue;
        uint64_t tx = rd<uint64_t>(m8 + 48);
        if (!best || tx > best_tx) { best = m8; best_tx = tx; }
    }
    if (!best) return fail(db, "no valid bbolt meta page");
    db->page_size = rd<uint32_t>(best + 8);
    const uint8_t* root = page_at(db, rd<uint64_t>(best + 16));
    if (!root) return fail(db, "root bucket page out of range");
    int r = find_bucket(db, root, "beacons", 0);
    if (r < 0) return -1;
    if (r > 0) return fail(db, "bucket \"beacons\" not found");
    if (db->bucket_root) {
        const uint8_t* bp = page_at(db, db->bucket_root);
        if (!bp) return fail(db, "beacons bucket root out of range");
        if (walk(db, bp, db->base + db->size, db->entries, 0)) return -1;
    } else {
        if (walk(db, db->inline_page, db->inline_end, db->entries, 0)) return -1;
    }
    return 0;
}

int64_t dl_count(const dl_db* db) { return db ? int64_t(db->entries.size()) : -1; }

}  // extern "C"

namespace {

// Decode entries [lo, hi) into row i - start; returns the first failing entry index or -1.
long decode_range(dl_db* db, size_t start, size_t lo, size_t hi, uint64_t* rounds, uint8_t* prev96,
                  uint8_t* prev_len, uint8_t* sigs96, uint8_t* sig_len, uint8_t* sigs_v2_96, uint8_t* v2_len,
                  std::string& err) {
    uint8_t scratch[96];
    for (size_t j = lo; j < hi; j++) {
        size_t i = j - start;
        const Entry& en = db->entries[j];
        Fields f;
        uint8_t* v2 = sigs_v2_96 ? sigs_v2_96 + 96 * i : scratch;
        std::memset(prev96 + 96 * i, 0, 96);
        std::memset(sigs96 + 96 * i, 0, 96);
        if (sigs_v2_96) std::memset(v2, 0, 96);
        if (parse_beacon(en.v, en.vs, f, prev96 + 96 * i, sigs96 + 96 * i, v2)) {
            err = "malformed beacon JSON at entry " + std::to_string(j);
            return long(j);
        }
        if (en.ks != 8) {
            err = "key is not an 8-byte round at entry " + std::to_string(j);
            return long(j);
        }
        uint64_t key = 0;
        for (int b = 0; b < 8; b++) key = key << 8 | en.k[b];
        if (key != f.round) {
            err = "key round " + std::to_string(key) + " != value round " + std::to_string(f.round);
            return long(j);
        }
        rounds[i] = f.round;
        // lengths above 96 are reported as 255 ("not a signature"); the bytes kept are the first 96
        prev_len[i] = uint8_t(f.prev_len > 96 ? 255 : f.prev_len);
        sig_len[i] = uint8_t(f.sig_len > 96 ? 255 : f.sig_len);
        if (v2_len) v2_len[i] = uint8_t(f.v2_len > 96 ? 255 : f.v2_len);
    }
    return -1;
}

}  // namespace

extern "C" {

int dl_load(dl_db* db, size_t start, size_t max_n, uint64_t* rounds, uint8_t* prev96, uint8_t* prev_len,
            uint8_t* sigs96, uint8_t* sig_len, uint8_t* sigs_v2_96, uint8_t* v2_len, size_t* n_out) {
    if (!db || !n_out || !rounds || !prev96 || !prev_len || !sigs96 || !sig_len) return -1;
    *n_out = 0;
    if (start > db->entries.size()) return fail(db, "start beyond the last entry");
    size_t n = std::min(max_n, db->entries.size() - start);
    // The values are independent: decode in parallel, contiguous slices per thread (the mmap'd
    // pages are read once; the SoA rows each thread writes are disjoint).
    unsigned hw = std::thread::hardware_concurrency();
    size_t nt = std::max<size_t>(1, std::min<size_t>({size_t(hw ? hw : 1), 16, (n + 16383) / 16384}));
    if (const char* e = std::getenv("DL_THREADS")) nt = std::max<size_t>(1, size_t(std::atoi(e)));
    std::vector<long> bad(nt, -1);
    std::vector<std::string> errs(nt);
    std::vector<std::thread> pool;
    size_t per = (n + nt - 1) / nt;
    for (size_t t = 0; t < nt; t++) {
        size_t lo = start + std::min(n, t * per), hi = start + std::min(n, (t + 1) * per);
        auto job = [=, &bad, &errs] {
            bad[t] = decode_range(db, start, lo, hi, rounds, prev96, prev_len, sigs96, sig_len, sigs_v2_96, v2_len,
                                  errs[t]);
        };
        if (nt == 1) job(); else pool.emplace_back(job);
    }
    for (auto& th : pool) th.join();
    for (size_t t = 0; t < nt; t++)
        if (bad[t] >= 0) return fail(db, errs[t]);   // lowest slice first = lowest failing entry
    *n_out = n;
    return 0;
}

const char* dl_last_error(const dl_db* db) { return db ? db->err.c_str() : "null handle"; }

void dl_close(dl_db* db) {
    if (!db) return;
    if (db->base) munmap(const_cast<uint8_t*>(db->base), db->size);
    if (db->fd >= 0) ::close(db->fd);
    delete db;
}

}  // extern "C"
