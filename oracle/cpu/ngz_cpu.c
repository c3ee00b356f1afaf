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
 *   NetFlowV9Packet::parse   netflow.rs:56-114 (count-driven set loop, InvalidCount),
 *                            Set::parse :143-235 (exact record length, per-record
 *                            processed_count, zero padding), templates :265-353,
 *                            ScopeField :443-475
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

typedef struct { int16_t ie; uint16_t len; uint8_t scope; } Spec;  /* scope: NFv9 ScopeIE code (1..5), 0 = IE */
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
    if (s->scope) {  /* NFv9 ScopeField (netflow.rs:443-475) */
        if (len > rem) return -1;
        if (s->scope <= 3) {  /* System / Interface / LineCard: reduced u32 */
            if (len > 4) return -1;
            f->tag = DT_unsigned32;
            f->v.u = be(p, len);
            return len;
        }
        f->tag = DT_octetArray;  /* Cache / Template / Unknown: raw bytes */
        f->len = (uint32_t)len;
        f->v.bytes = (uint8_t *)malloc(len ? len : 1);
        memcpy(f->v.bytes, p, len);
        return len;
    }
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
    case DT_dtMs:  /* chrono timestamp_millis_opt range (0.4.45) */
        if (len != 8 || rem < 8) return -1;
        f->v.u = be(p, 8);
        if ((int64_t)f->v.u < -8334601315200000LL || (int64_t)f->v.u > 8210266876799999LL) return -1;
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
    uint32_t n_pre;  /* messages [0, n_pre) (the exporter's templates) are decoded by every thread first */
    uint64_t records, errors;
    uint64_t *sums;  /* per field index, wrapping sum of canonical u64 values */
    int nsums;
} Job;

typedef struct { Field *fields; int n; } Record;
typedef struct { Record *recs; size_t n, cap; } Records;

static void push_record(Records *rs, Record r) {
    if (rs->n == rs->cap) { rs->cap = rs->cap ? rs->cap * 2 : 64; rs->recs = (Record *)realloc(rs->recs, rs->cap * sizeof(Record)); }
    rs->recs[rs->n++] = r;
}

static void put_template(Template **tmap, uint32_t tid, Template *t) {
    if (tmap[tid]) { free(tmap[tid]->specs); free(tmap[tid]); }
    tmap[tid] = t;
}

/* FieldSpecifier::parse (deserializer/mod.rs:53-66); 0 = ok */
static int parse_spec(const uint8_t *b, uint32_t bl, uint32_t *q, Spec *sp) {
    if (bl - *q < 4) return -1;
    uint32_t code = (uint32_t)be(b + *q, 2), fl = (uint32_t)be(b + *q + 2, 2);
    *q += 4;
    uint32_t pen = 0;
    if (code & 0x8000) { if (bl - *q < 4) return -1; pen = (uint32_t)be(b + *q, 4); *q += 4; code &= 0x7FFF; }
    int ie = ie_lookup(pen, (uint16_t)code);
    if (ie == -1) return -1;  /* UndefinedIANAIE */
    sp->ie = (int16_t)(ie < 0 ? -1 : ie);
    sp->len = (uint16_t)fl;
    sp->scope = 0;
    return 0;
}

/* DataRecord::parse of one record at b[*q..bl) (ipfix.rs:335-370 / netflow.rs:399-432) */
static int parse_record(const uint8_t *b, uint32_t bl, uint32_t *q, const Template *t, Records *rs) {
    Record r;
    r.n = t->n;
    r.fields = (Field *)malloc(sizeof(Field) * (t->n ? t->n : 1));  /* Box<[Field]> */
    int ok = 1;
    for (int i = 0; i < t->n; ++i) {
        int c = parse_field(b + *q, (int)(bl - *q), &t->specs[i], &r.fields[i]);
        if (c < 0) { ok = 0; r.n = i; break; }
        *q += (uint32_t)c;
    }
    push_record(rs, r);
    return ok;
}

static int ipfix_message(const uint8_t *p, uint32_t len, Template **tmap, Records *rs) {
    uint32_t pos = 16;
    while (pos < len) {
        if (len - pos < 4) return 0;
        uint32_t id = (uint32_t)be(p + pos, 2), sl = (uint32_t)be(p + pos + 2, 2);
        if ((id != 2 && id != 3 && id < 256) || sl < 4 || sl > len - pos) return 0;
        const uint8_t *b = p + pos + 4;
        uint32_t bl = sl - 4, q = 0;
        if (id == 2 || id == 3) {  /* (options) template sets, ipfix.rs:162-181,276-327,384-413 */
            while (id == 2 ? q < bl : bl - q > 3) {
                if (bl - q < 4) return 0;
                uint32_t tid = (uint32_t)be(b + q, 2), total = (uint32_t)be(b + q + 2, 2), scount = 0;
                q += 4;
                if (tid < 256) return 0;
                if (id == 3) { if (bl - q < 2) return 0; scount = (uint32_t)be(b + q, 2); q += 2; if (scount > total) return 0; }
                Template *t = (Template *)calloc(1, sizeof(Template));
                t->specs = (Spec *)calloc(total ? total : 1, sizeof(Spec));
                t->n = (int)total;
                for (uint32_t i = 0; i < total; ++i) {
                    if (parse_spec(b, bl, &q, &t->specs[i])) { free(t->specs); free(t); return 0; }
                    t->minlen += t->specs[i].len == 0xFFFF ? 1 : (int)t->specs[i].len;
                }
                put_template(tmap, tid, t);
            }
            for (; id == 3 && q < bl; ++q) if (b[q]) return 0;  /* options padding must be zero */
        } else {
            Template *t = tmap[id];
            if (!t) return 0;
            while (t->minlen > 0 && bl - q >= (uint32_t)t->minlen)  /* ipfix.rs:219-222 */
                if (!parse_record(b, bl, &q, t, rs)) return 0;
            t->processed++;  /* once per set (ipfix.rs:223) */
        }
        pos += sl;
    }
    return 1;
}

static int nfv9_message(const uint8_t *p, uint32_t dl, Template **tmap, Records *rs) {
    if (dl < 20) return 0;
    uint32_t count = (uint32_t)be(p + 2, 2), i = count, pos = 20;
    while (i > 0 && dl - pos > 3) {  /* netflow.rs:89 */
        uint32_t id = (uint32_t)be(p + pos, 2), sl = (uint32_t)be(p + pos + 2, 2);
        if ((id != 0 && id != 1 && id < 256) || sl < 4 || sl > dl - pos) return 0;
        const uint8_t *b = p + pos + 4;
        uint32_t bl = sl - 4, q = 0;
        if (id == 0) {  /* template set, netflow.rs:324-353 */
            while (q < bl) {
                if (bl - q < 4) return 0;
                uint32_t tid = (uint32_t)be(b + q, 2), cnt = (uint32_t)be(b + q + 2, 2);
                q += 4;
                if (tid < 256) return 0;
                Template *t = (Template *)calloc(1, sizeof(Template));
                t->specs = (Spec *)calloc(cnt ? cnt : 1, sizeof(Spec));
                t->n = (int)cnt;
                for (uint32_t k = 0; k < cnt; ++k) {
                    if (parse_spec(b, bl, &q, &t->specs[k])) { free(t->specs); free(t); return 0; }
                    t->minlen += (int)t->specs[k].len;  /* exact record length, 65535 literal */
                }
                put_template(tmap, tid, t);
            }
            i -= 1;
        } else if (id == 1) {  /* options template set, netflow.rs:265-310 */
            while (bl - q > 3) {
                if (bl - q < 6) return 0;
                uint32_t tid = (uint32_t)be(b + q, 2), slen = (uint32_t)be(b + q + 2, 2), olen = (uint32_t)be(b + q + 4, 2);
                q += 6;
                if (tid < 256 || slen > bl - q || olen > bl - q - slen) return 0;
                uint32_t n = slen / 4 + olen / 4;
                Template *t = (Template *)calloc(1, sizeof(Template));
                t->specs = (Spec *)calloc(n ? n : 1, sizeof(Spec));
                uint32_t se = q + slen, oe = se + olen;
                while (q < se) {  /* ScopeFieldSpecifier (netflow.rs:368-388) */
                    if (se - q < 4) { free(t->specs); free(t); return 0; }
                    uint32_t code = (uint32_t)be(b + q, 2), fl = (uint32_t)be(b + q + 2, 2);
                    q += 4;
                    if (code & 0x8000) { q += 4; code = 0; }  /* enterprise scope: raw bytes */
                    Spec *sp = &t->specs[t->n++];
                    sp->ie = -1; sp->len = (uint16_t)fl; sp->scope = (uint8_t)(code >= 1 && code <= 5 ? code : 4);
                    t->minlen += (int)fl;
                }
                while (q < oe) {
                    if (parse_spec(b, oe, &q, &t->specs[t->n])) { free(t->specs); free(t); return 0; }
                    t->minlen += (int)t->specs[t->n++].len;
                }
                put_template(tmap, tid, t);
            }
            for (; q < bl; ++q) if (b[q]) return 0;
            i -= 1;
        } else {
            Template *t = tmap[id];
            if (!t) return 0;
            uint32_t nrec = 0;
            if (t->minlen)
                while (bl - q >= (uint32_t)t->minlen) {
                    if (!parse_record(b, bl, &q, t, rs)) return 0;
                    t->processed++;  /* per record (netflow.rs:218) */
                    ++nrec;
                }
            for (; q < bl; ++q) if (b[q]) return 0;  /* check_padding_value */
            if (nrec > i) return 0;                   /* InvalidCount */
            i -= nrec;
        }
        pos += sl;
    }
    return 1;
}

static void decode_message(const uint8_t *p, uint32_t dl, Template **tmap, Job *job) {
    /* FlowInfoCodec::decode gate and dispatch (codec.rs:189-220) */
    if (dl < 16) return;
    uint32_t ver = (uint32_t)be(p, 2), len = (uint32_t)be(p + 2, 2);
    if (dl < len) return;
    /* the parsed packet owns its records until it is dropped */
    Records rs = {NULL, 0, 0};
    int ok;
    if (ver == 10) ok = len >= 16 && ipfix_message(p, len, tmap + 0, &rs);
    else if (ver == 9) ok = nfv9_message(p, dl, tmap + 65536, &rs);
    else ok = 0;
    if (ok) {
        job->records += rs.n;
        for (size_t k = 0; k < rs.n; ++k)
            for (int i = 0; i < rs.recs[k].n && i < job->nsums; ++i) {
                const Field *f = &rs.recs[k].fields[i];
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
    for (size_t k = 0; k < rs.n; ++k) {
        for (int i = 0; i < rs.recs[k].n; ++i) free_field(&rs.recs[k].fields[i]);
        free(rs.recs[k].fields);
    }
    free(rs.recs);
}

static void *run(void *arg) {
    Job *job = (Job *)arg;
    /* per-peer codec: the IPFIX TemplatesMap [0, 65536) and the NFv9 one [65536, 131072) */
    Template **tmap = (Template **)calloc(2 * 65536, sizeof(Template *));
    for (uint32_t i = 0; i < job->n_pre; ++i) decode_message(job->bytes + job->offs[i], job->lens[i], tmap, job);
    job->records = 0;
    job->errors = 0;
    for (int i = 0; i < job->nsums; ++i) job->sums[i] = 0;
    for (uint32_t i = job->first; i < job->last; ++i)
        decode_message(job->bytes + job->offs[i], job->lens[i], tmap, job);
    for (int i = 0; i < 2 * 65536; ++i)
        if (tmap[i]) { free(tmap[i]->specs); free(tmap[i]); }
    free(tmap);
    return NULL;
}

/* Decode messages [n_pre, n) on `threads` threads, each an independent codec
 * (one exporter peer per thread, as collector actors partition peers) over a
 * contiguous message range, after decoding the template messages [0, n_pre)
 * itself.  Returns records decoded; sums[nsums] (optional) receive per-field
 * wrapping sums of the canonical values; *errors the failed messages. */
uint64_t ngz_cpu_decode(const uint8_t *bytes, const uint64_t *offs, const uint32_t *lens, uint32_t n,
                        uint32_t n_pre, int threads, uint64_t *sums, int nsums, uint64_t *errors) {
    if (threads < 1) threads = 1;
    if (n_pre > n) n_pre = n;
    pthread_t *th = (pthread_t *)calloc((size_t)threads, sizeof(pthread_t));
    Job *jobs = (Job *)calloc((size_t)threads, sizeof(Job));
    const uint32_t m = n - n_pre;
    for (int t = 0; t < threads; ++t) {
        jobs[t].bytes = bytes; jobs[t].offs = offs; jobs[t].lens = lens;
        jobs[t].first = n_pre + (uint32_t)((uint64_t)m * t / threads);
        jobs[t].last = n_pre + (uint32_t)((uint64_t)m * (t + 1) / threads);
        jobs[t].n_pre = n_pre;
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
