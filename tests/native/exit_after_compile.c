/* A plain C host of libngz that exits with background kernel compiles in
 * flight, without calling ngz_rtc_drain: it decodes one batch that defines
 * four templates (each starts a hiprtc compile on a background thread and is
 * decoded by the generic kernel meanwhile), destroys its context and returns
 * from main.  ngz_ctx_destroy must join those compiles (synchronous drop, as
 * the reference codec's, crates/flow-pkt/src/codec.rs:68-82), so the process
 * exits 0 instead of hanging in the compiler's exit-time destructors.
 *
 * Prints "compiling=<n> records=<r>": n = slots decoded by the generic kernel
 * while their own kernel compiled (ngz_slot_kernel == 2) when the context was
 * destroyed.  Used by tests/test_gpu_rtc.py (built by __graft_entry__.build). */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "ngz/flow_decode.h"

#define N_TEMPLATES 4
#define RECORDS_PER_MSG 200
#define MSGS_PER_TEMPLATE 2

static uint8_t buf[1 << 20];
static size_t used;

static void put16(uint8_t *p, uint32_t v) { p[0] = (uint8_t)(v >> 8); p[1] = (uint8_t)v; }
static void put32(uint8_t *p, uint32_t v) { put16(p, v >> 16); put16(p + 2, v & 0xFFFF); }

/* (IE id, length) of template k: an IPv4 5-tuple + counters, then k extra ipClassOfService bytes so
 * that every template has its own layout (its own compile) */
static int template_fields(int k, uint16_t ids[], uint16_t lens[]) {
    static const uint16_t base_id[] = {8, 12, 7, 11, 4, 1, 2};
    static const uint16_t base_len[] = {4, 4, 2, 2, 1, 8, 8};
    int n = 0;
    for (int i = 0; i < 7; ++i, ++n) { ids[n] = base_id[i]; lens[n] = base_len[i]; }
    for (int i = 0; i <= k; ++i, ++n) { ids[n] = 5; lens[n] = 1; }
    return n;
}

static uint8_t *msg_begin(uint32_t seq) {
    uint8_t *m = buf + used;
    put16(m, 10);
    put32(m + 4, 1700000000u);
    put32(m + 8, seq);
    put32(m + 12, 1);
    used += 16;
    return m;
}

static void msg_end(uint8_t *m) { put16(m + 2, (uint32_t)(buf + used - m)); }

int main(void) {
    uint64_t offs[1 + N_TEMPLATES * MSGS_PER_TEMPLATE];
    uint32_t lens[1 + N_TEMPLATES * MSGS_PER_TEMPLATE];
    uint32_t n = 0, seq = 0;
    uint16_t ids[16], flen[16];

    /* one message with the four template sets */
    uint8_t *m = msg_begin(seq);
    for (int k = 0; k < N_TEMPLATES; ++k) {
        const int nf = template_fields(k, ids, flen);
        uint8_t *s = buf + used;
        put16(s, 2);
        put16(s + 4, 256 + k);
        put16(s + 6, nf);
        used += 8;
        for (int f = 0; f < nf; ++f, used += 4) { put16(buf + used, ids[f]); put16(buf + used + 2, flen[f]); }
        put16(s + 2, (uint32_t)(buf + used - s));
    }
    msg_end(m);
    offs[n] = (uint64_t)(m - buf); lens[n] = (uint32_t)(buf + used - m); ++n;

    /* data messages */
    uint64_t x = 0x4E475A4500000006ull;
    for (int k = 0; k < N_TEMPLATES; ++k) {
        const int nf = template_fields(k, ids, flen);
        uint32_t rl = 0;
        for (int f = 0; f < nf; ++f) rl += flen[f];
        for (int j = 0; j < MSGS_PER_TEMPLATE; ++j) {
            m = msg_begin(seq);
            uint8_t *s = buf + used;
            put16(s, 256 + k);
            used += 4;
            for (uint32_t r = 0; r < RECORDS_PER_MSG * rl; ++r) {
                x = x * 6364136223846793005ull + 1442695040888963407ull;
                buf[used++] = (uint8_t)(x >> 56);
            }
            put16(s + 2, (uint32_t)(buf + used - s));
            msg_end(m);
            seq += RECORDS_PER_MSG;
            offs[n] = (uint64_t)(m - buf); lens[n] = (uint32_t)(buf + used - m); ++n;
        }
    }

    if (ngz_abi_version() != NGZ_ABI_VERSION) { fprintf(stderr, "libngz ABI mismatch\n"); return 2; }
    ngz_ctx *ctx = NULL;
    if (ngz_ctx_create(0, &ctx) != NGZ_OK) { fprintf(stderr, "ngz_ctx_create failed\n"); return 3; }
    ngz_batch_out out;
    if (ngz_decode_batch_host(ctx, buf, used, offs, lens, n, &out) != NGZ_OK) {
        fprintf(stderr, "decode failed: %s\n", ngz_last_error(ctx));
        return 4;
    }
    int compiling = 0;
    uint64_t records = 0;
    for (uint32_t s = 0; s < out.n_slots; ++s) {
        compiling += ngz_slot_kernel(ctx, s) == 2;
        records += out.slots[s].n_records;
    }
    printf("compiling=%d records=%llu\n", compiling, (unsigned long long)records);
    fflush(stdout);
    ngz_ctx_destroy(ctx);
    return 0; /* no ngz_rtc_drain: the destroy must have joined the compiles */
}
