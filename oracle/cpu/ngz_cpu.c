/*
 * CPU ORACLE / BASELINE — test and benchmark infrastructure only, never part
 * of the product path (netgauze_amd/ does not link or load this).
 *
 * Plain-C restatement of the reference's record-at-a-time IPFIX decode, used
 * as (a) the bench's cpu_baseline ("port": the Rust reference cannot be built
 * or run here) and (b) a large-size checker (per-field sums
 * compared with the GPU columns).  It follows:
 *   IpfixPacket::parse       crates/flow-pkt/src/wire/deserializer/ipfix.rs:54-104
 *   Set::parse               ipfix.rs:133-238 (templates, data sets, min length)
 *   TemplateRecord::parse    ipfix.rs:384-413, FieldSpecifier::parse mod.rs:53-66
 *   DataRecord::parse        ipfix.rs:335-370: one heap-allocated Field array
 *                            per record (Box<[Field]>), per-field dispatch on
 *                            the IE (the generated match, generator.rs:2959-2978)
 *   Field::parse rules       generator.rs:1439-1807 (reduced-size ints, bytes,
 *                            vlen prefixes, tcpControlBits truncation)
 * Records are freed when their message is dropped, as the Rust packet is.
 * Pinned: tests/test_cpu_port.py checks its per-field sums against the Python
 * oracle (itself pinned byte-exact to the reference's golden JSON).
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

enum { DT_octetArray = 0, DT_unsigned8, DT_unsigned16, DT_unsigned32, DT_unsigned64, DT_signed8, DT_signed16,
       DT_signed32, DT_signed64, DT_float32, DT_float64, DT_boolean, DT_macAddress, DT_string, DT_dtSec,
       DT_dtMs, DT_dtUs, DT_dtNs, DT_ipv4, DT_ipv6, DT_basicList, DT_subTemplateList, DT_subTemplateMultiList,
       DT_unsigned256 };

typedef struct { uint32_t pen; uint16_t id; uint8_t dt; uint8_t flags; const char *name; } IeRow;
#define NGZ_IE(pen, id, dt, fl, nm) {pen, (uint16_t)(id), (uint8_t)(dt), (uint8_t)(fl), nm},
#define NGZ_VENDOR(pen, nm)
static const IeRow kIes[] = {
#include "../../netgauze_amd/csrc/ie_table.inc"
};
#undef NGZ_IE
#undef NGZ_VENDOR

/* the Rust Field enum: tag + payload (24 bytes) */
typedef struct {
    uint16_t ie;       /* index into kIes, or 0xFFFF unknown */
    uint8_t tag;       /* data type */
    uint8_t pad;
    uint32_t len;
    union { uint64_t u; int64_t i; uint8_t *bytes; uint8_t small[16]; } v;
} Field;

typedef struct { int16_t ie; uint16_t len; } Spec;
typedef struct { int n; Spec *specs; int minlen; uint64_t processed; } Template;

static int ie_lookup(uint32_t pen, uint16_t id) {
    /* registry index (linear probe table built once) */
    static int built = 0;
    static int32_t tab[1 << 16];
    static pthread_mutex_t mu = PTHREAD_MUTEX_INITIALIZER;
    if (!built) {
        pthread_mutex_lock(&mu);
        if (!built) {
            for (int i = 0; i < (1 << 16); ++i) tab[i] = -1;
            for (int i = 0; i < (int)(sizeof kIes / sizeof kIes[0]); ++i)
                if (kIes[i].pen == 0) tab[kIes[i].id] = i;
            built = 1;
        }
        pthread_mutex_unlock(&mu);
    }
    if (pen != 0) {
        for (int i = 0; i < (int)(sizeof kIes / sizeof kIes[0]); ++i)
            if (kIes[i].pen == pen && kIes[i].id == (id & 0x7FFF)) return i;
        return -2;  /* vendor unknown / unknown PEN: raw bytes */
    }
    return tab[id];
}

static inline uint64_t be(const uint8_t *p, int n) {
    uint64_t v = 0;
    for (int i = 0; i < n; ++i) v = (v << 8) | p[i];
    return v;
}

/* Field::parse; returns bytes consumed or -1 */
static int parse_field(const uint8_t *p, int rem, const Spec *s, Field *f) {
    int len = s->len;
    f->ie = (uint16_t)s->ie;
    int dt = s->ie >= 0 ? kIes[s->ie].dt : DT_octetArray;
    f->tag = (uint8_t)dt;
    int hdr = 0;
    switch (dt) {
    case DT_unsigned8: case DT_unsigned16: case DT_unsigned32: case DT_unsigned64:
    case DT_ipv4: case DT_dtSec: case DT_float64: case DT_boolean:
        if (len > rem || len > 8) return -1;
        f->v.u = be(p, len);
        if (s->ie >= 0 && (kIes[s->ie].flags & 2)) f->v.u &= 0xFF; /* tcpControlBits */
        if (dt == DT_boolean) f->v.u = f->v.u != 0;
        return len;
    case DT_signed32: {
        if (len > rem || len > 4) return -1;
        uint64_t u = be(p, len);
        int sh = len ? 64 - 8 * len : 0;
        f->v.i = ((int64_t)(u << sh)) >> sh;
        return len;
    }
    case DT_dtMs:
        if (len != 8 || rem < 8) return -1;
        f->v.u = be(p, 8);
        return 8;
    case DT_dtUs: case DT_dtNs: {
        if (len != 8 || rem < 8) return -1;
        uint32_t secs = (uint32_t)be(p, 4), frac = (uint32_t)be(p + 4, 4);
        uint32_t ns = (uint32_t)(1000000000.0 * ((double)frac / 4294967295.0));
        if (ns >= 1000000000u && secs % 60 != 59) return -1;
        f->v.u = (uint64_t)secs | ((uint64_t)ns << 32);
        return 8;
    }
    case DT_macAddress: case DT_ipv6: case DT_unsigned256:
        if (len > rem || len > 16 + 16) return -1;
        f->len = (uint32_t)len;
        if (len <= 16) memcpy(f->v.small, p, len);
        else { f->v.bytes = (uint8_t *)malloc(len); memcpy(f->v.bytes, p, len); }
        return len;
    default: {  /* octetArray / string / lists / unknown: vlen-aware raw bytes */
        if (len == 0xFFFF) {
            if (rem < 1) return -1;
            int sl = p[0];
            hdr = 1;
            if (sl == 0xFF) { if (rem < 4) return -1; sl = (int)be(p + 1, 3); hdr = 4; }
            len = sl;
        }
        if (hdr + len > rem) return -1;
        f->len = (uint32_t)len;
        f->v.bytes = (uint8_t *)malloc(len ? len : 1);  /* Box<[u8]> / Box<str> */
        memcpy(f->v.bytes, p + hdr, len);
        return hdr + len;
    }
    }
}

static void free_field(Field *f) {
    int dt = f->tag;
    if ((dt == DT_macAddress || dt == DT_ipv6 || dt == DT_unsigned256) && f->len <= 16) return;
    if (dt == DT_octetArray || dt == DT_string || dt == DT_basicList || dt == DT_subTemplateList ||
        dt == DT_subTemplateMultiList || dt == DT_macAddress || dt == DT_ipv6 || dt == DT_unsigned256)
        free(f->v.bytes);
}

typedef struct {
    const uint8_t *bytes;
    const uint64_t *offs;
    const uint32_t *lens;
    uint32_t first, last;
    const uint8_t *tmpl;  /* template message prepended to every thread's stream */
    uint32_t tmpl_len;
    uint64_t records, errors;
    uint64_t *sums;  /* per field index, wrapping sum of canonical u64 values */
    int nsums;
} Job;

typedef struct { Field *fields; int n; } Record;

static void decode_message(const uint8_t *p, uint32_t dl, Template **tmap, Job *job) {
    if (dl < 16) return;
    uint32_t ver = (uint32_t)be(p, 2), len = (uint32_t)be(p + 2, 2);
    if (dl < len || ver != 10 || len < 16) { job->errors++; return; }
    /* the parsed packet owns its records until it is dropped */
    Record *recs = NULL;
    size_t nrec = 0, cap = 0;
    uint32_t pos = 16;
    int ok = 1;
    while (pos < len && ok) {
        if (len - pos < 4) { ok = 0; break; }
        uint32_t id = (uint32_t)be(p + pos, 2), sl = (uint32_t)be(p + pos + 2, 2);
        if ((id != 2 && id != 3 && id < 256) || sl < 4 || sl > len - pos) { ok = 0; break; }
        const uint8_t *b = p + pos + 4;
        uint32_t bl = sl - 4;
        if (id == 2) {
            uint32_t q = 0;
            while (q < bl) {
                if (bl - q < 4) { ok = 0; break; }
                uint32_t tid = (uint32_t)be(b + q, 2), cnt = (uint32_t)be(b + q + 2, 2);
                q += 4;
                Template *t = (Template *)calloc(1, sizeof(Template));
                t->specs = (Spec *)calloc(cnt ? cnt : 1, sizeof(Spec));
                t->n = (int)cnt;
                for (uint32_t i = 0; i < cnt; ++i) {
                    if (bl - q < 4) { ok = 0; break; }
                    uint32_t code = (uint32_t)be(b + q, 2), fl = (uint32_t)be(b + q + 2, 2);
                    q += 4;
                    uint32_t pen = 0;
                    if (code & 0x8000) { pen = (uint32_t)be(b + q, 4); q += 4; code &= 0x7FFF; }
                    int ie = ie_lookup(pen, (uint16_t)code);
                    if (ie == -1) { ok = 0; break; }
                    t->specs[i].ie = (int16_t)(ie < 0 ? -1 : ie);
                    t->specs[i].len = (uint16_t)fl;
                    t->minlen += fl == 0xFFFF ? 1 : (int)fl;
                }
                if (!ok) { free(t->specs); free(t); break; }
                if (tmap[tid]) { free(tmap[tid]->specs); free(tmap[tid]); }
                tmap[tid] = t;
            }
        } else if (id == 3) {
            /* options templates are not part of the baseline workload */
        } else {
            Template *t = tmap[id];
            if (!t) { ok = 0; break; }
            uint32_t q = 0;
            while (t->minlen > 0 && bl - q >= (uint32_t)t->minlen) {
                Record r;
                r.n = t->n;
                r.fields = (Field *)malloc(sizeof(Field) * (t->n ? t->n : 1));  /* Box<[Field]> */
                for (int i = 0; i < t->n; ++i) {
                    int c = parse_field(b + q, (int)(bl - q), &t->specs[i], &r.fields[i]);
                    if (c < 0) { ok = 0; r.n = i; break; }
                    q += (uint32_t)c;
                }
                if (nrec == cap) { cap = cap ? cap * 2 : 64; recs = (Record *)realloc(recs, cap * sizeof(Record)); }
                recs[nrec++] = r;
                if (!ok) break;
            }
            t->processed++;
        }
        pos += sl;
    }
    if (ok) {
        job->records += nrec;
        for (size_t k = 0; k < nrec; ++k)
            for (int i = 0; i < recs[k].n && i < job->nsums; ++i) {
                const Field *f = &recs[k].fields[i];
                uint64_t v = 0;
                if (f->tag == DT_octetArray || f->tag == DT_string || f->tag >= DT_basicList ||
                    f->tag == DT_macAddress || f->tag == DT_ipv6) {
                    const uint8_t *src = (f->tag == DT_macAddress || f->tag == DT_ipv6) ? f->v.small : f->v.bytes;
                    for (uint32_t j = 0; j < f->len; ++j) v = v * 131 + src[j];
                } else {
                    v = f->v.u;
                }
                job->sums[i] += v;
            }
    } else {
        job->errors++;
    }
    for (size_t k = 0; k < nrec; ++k) {
        for (int i = 0; i < recs[k].n; ++i) free_field(&recs[k].fields[i]);
        free(recs[k].fields);
    }
    free(recs);
}

static void *run(void *arg) {
    Job *job = (Job *)arg;
    Template **tmap = (Template **)calloc(65536, sizeof(Template *));  /* per-peer TemplatesMap */
    if (job->tmpl) decode_message(job->tmpl, job->tmpl_len, tmap, job);
    for (uint32_t i = job->first; i < job->last; ++i)
        decode_message(job->bytes + job->offs[i], job->lens[i], tmap, job);
    for (int i = 0; i < 65536; ++i)
        if (tmap[i]) { free(tmap[i]->specs); free(tmap[i]); }
    free(tmap);
    return NULL;
}

/* Decode messages [0, n) on `threads` threads, each an independent codec over
 * a contiguous message range (one exporter peer per thread, as collector
 * actors partition peers).  Returns records decoded; sums[nsums] (optional)
 * receive per-field wrapping sums of the canonical values. */
uint64_t ngz_cpu_decode(const uint8_t *bytes, const uint64_t *offs, const uint32_t *lens, uint32_t n,
                        const uint8_t *tmpl, uint32_t tmpl_len, int threads, uint64_t *sums, int nsums,
                        uint64_t *errors) {
    if (threads < 1) threads = 1;
    pthread_t *th = (pthread_t *)calloc((size_t)threads, sizeof(pthread_t));
    Job *jobs = (Job *)calloc((size_t)threads, sizeof(Job));
    for (int t = 0; t < threads; ++t) {
        jobs[t].bytes = bytes; jobs[t].offs = offs; jobs[t].lens = lens;
        jobs[t].first = (uint32_t)((uint64_t)n * t / threads);
        jobs[t].last = (uint32_t)((uint64_t)n * (t + 1) / threads);
        jobs[t].tmpl = tmpl; jobs[t].tmpl_len = tmpl_len;
        jobs[t].nsums = nsums;
        jobs[t].sums = (uint64_t *)calloc(nsums > 0 ? (size_t)nsums : 1, 8);
        pthread_create(&th[t], NULL, run, &jobs[t]);
    }
    uint64_t total = 0, errs = 0;
    for (int t = 0; t < threads; ++t) {
        pthread_join(th[t], NULL);
        total += jobs[t].records;
        errs += jobs[t].errors;
        for (int i = 0; i < nsums; ++i) sums[i] += jobs[t].sums[i];
        free(jobs[t].sums);
    }
    if (errors) *errors = errs;
    free(th);
    free(jobs);
    return total;
}
