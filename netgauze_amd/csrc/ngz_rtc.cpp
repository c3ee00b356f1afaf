// Per-template decode kernels, generated and compiled at run time (hiprtc).
//
// A template's decode plan (DevPlan: record length + per-field offset,
// length, column width, decode kind) is turned into HIP source in which every
// field is a constant: the generated kernel walks only that template's chunks
// and, per 64-record pass, loads exactly the record dwords its fields touch
// into VGPRs (statically planned 80-byte windows), then extracts, byte-swaps,
// widens and stores each field with constant register indices and shifts.
// It is the north star's "one kernel specialised per active template ID";
// the generic field-table kernel (ngz_kernels.hip) decodes the same plans and
// is used when specialisation is off or a compile fails.
//
// Kernels are cached process-wide by (device, plan signature): every template
// with the same layout -- the same template re-announced by an exporter, or
// the same layout on another exporter peer -- shares one code object.
//
// Compiles are off the decode path: ngz_rtc_kernel_async starts generate +
// hiprtc + module load on a background thread and returns at once; the
// context decodes that template with the generic kernel until the entry is
// ready (ngz_rtc_poll).  The cache lock is held only for the map lookup, never
// across a compile, so a new template on one exporter's context never stalls
// another context.  Each entry compiles once; concurrent askers wait on it
// (ngz_rtc_kernel, synchronous) or poll it (async).
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <hip/hiprtc.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "ngz/flow_decode.h"
#include "ngz_internal.h"

namespace {

// texts of flow_decode.h, ngz_internal.h and ngz_dev.h (tools/embed_sources.py)
#include "ngz_rtc_sources.inc"

constexpr uint32_t kWinDw = 19;  // usable dwords of a register window (ngz_dev.h WIN_DW - 1)

struct Item {           // one extraction step of the generated pass body
    int type;           // 0 numeric, 1 raw piece, 2 string check (window), 3 string check (global), 4 fail
    uint32_t f, off, len, width, kind, col_off;
    uint32_t j, piece, pad_to;  // raw pieces
    uint32_t d0, d1;    // record dwords touched (inclusive), types 0-2
};

// Defines of the generated source from experiment knobs (NGZ_LD_AUX / NGZ_ST_AUX / NGZ_WIN_ROT; the
// experiment build only, ngz_dev.h)
std::string cpol_defines() {
    std::string s;
    for (const char *k : {"NGZ_LD_AUX", "NGZ_ST_AUX", "NGZ_WIN_ROT"})
        if (const int64_t v = ngz_knob(k, -1); v >= 0) s += std::string("#define ") + k + " " + std::to_string(v) + "\n";
    return s;
}

bool staged_rows(const DevPlan &P);

// The cache key covers every input generate() branches on: the kernel shape (staged_rows
// depends on the protocol, which the field list alone does not show) included.
std::string signature(const DevPlan &P) {
    std::string s = "rl" + std::to_string(P.rec_len) + "lw" + std::to_string(P.lds_waves) + "dm" +
                    std::to_string(P.reserved0) + (staged_rows(P) ? "sr" : "") + (P.has_vlen ? "v" : "");
    if (const int64_t v = ngz_knob("NGZ_LD_AUX", -1); v >= 0) s += "la" + std::to_string(v);
    if (const int64_t v = ngz_knob("NGZ_ST_AUX", -1); v >= 0) s += "sa" + std::to_string(v);
    if (const int64_t v = ngz_knob("NGZ_WIN_ROT", -1); v >= 0) s += "wr" + std::to_string(v);
    char b[96];
    for (uint32_t f = 0; f < P.n_fields; ++f) {
        const DevField &d = P.f[f];
        snprintf(b, sizeof b, ";%u,%u,%u,%u,%u,%u", d.off, d.len, d.width, d.kind, d.col_off, d.flags);
        s += b;
    }
    return s;
}

std::string generate_vlen(const DevPlan &P);

// The parts of a fixed template's generated decode: the pass body (register
// windows, extraction, column stores through ColT / ColGlb) and, when staged
// in LDS, the store step; rows per lane and layout; LDS waves and row bytes.
struct FixedParts {
    int rpl = 4;
    bool consec = true;
    uint32_t lw = 0, rowb = 0, rec_len = 0;
    std::string pass, store;
};

FixedParts fixed_parts(const DevPlan &P) {
    std::vector<Item> items;
    for (uint32_t f = 0; f < P.n_fields; ++f) {
        const DevField &d = P.f[f];
        Item it{};
        it.f = f;
        it.off = d.off;
        it.len = d.len;
        it.width = d.width;
        it.kind = d.kind;
        it.col_off = d.col_off;
        switch (d.kind) {
        case NGZ_K_FAIL:
            it.type = 4;
            items.push_back(it);
            break;
        case NGZ_K_UINT: case NGZ_K_SCOPE32: case NGZ_K_TCPFLAGS: case NGZ_K_SINT:
        case NGZ_K_BOOL: case NGZ_K_DTMS: case NGZ_K_DTFRAC: {
            uint32_t L = d.len;
            if (d.kind == NGZ_K_DTMS || d.kind == NGZ_K_DTFRAC) L = 8;
            if (d.kind == NGZ_K_BOOL) L = 1;
            if (L == 0) L = 1;
            it.type = 0;
            it.d0 = d.off >> 2;
            it.d1 = (d.off + L - 1) >> 2;
            items.push_back(it);
            break;
        }
        case NGZ_K_STR: case NGZ_K_BYTES: case NGZ_K_U256: {
            if (d.kind == NGZ_K_STR) {
                Item c = it;
                c.type = d.len <= 64 ? 2 : 3;
                c.d0 = d.off >> 2;
                c.d1 = d.len ? (d.off + d.len - 1) >> 2 : c.d0;
                items.push_back(c);
            }
            for (uint32_t j = 0;; j += 64) {
                Item r = it;
                r.type = 1;
                r.j = j;
                r.piece = std::min<uint32_t>(64, d.len - j);
                const bool last = j + 64 >= d.len;
                r.pad_to = last ? d.width : 0;
                r.d0 = (d.off + j) >> 2;
                r.d1 = r.piece ? (d.off + j + r.piece - 1) >> 2 : r.d0;
                items.push_back(r);
                if (last) break;
            }
            break;
        }
        default:
            break;  // vlen: not device-decodable (plan.rpl == 0 never reaches here)
        }
    }
    // windows: greedy in record order; a window spans <= kWinDw dwords
    std::vector<std::pair<uint32_t, uint32_t>> wins;  // (first dword, dword count)
    std::vector<int> item_win(items.size(), -1);
    for (size_t i = 0; i < items.size(); ++i) {
        const Item &it = items[i];
        if (it.type == 3 || it.type == 4) continue;
        if (wins.empty() || it.d0 < wins.back().first || it.d1 >= wins.back().first + kWinDw) wins.push_back({it.d0, 1});
        auto &w = wins.back();
        w.second = std::max(w.second, it.d1 - w.first + 1);
        item_win[i] = (int)wins.size() - 1;
    }
    // Rows per lane and their layout (NGZ_RTC_LAYOUT overrides for experiments):
    // "c4"/"c2" = 4/2 consecutive rows per lane, numeric columns packed into
    // one wide store per lane; "r1"/"r2"/"r4" = 1/2/4 rows per lane, 64 apart.
    // Default by record length (measured, profiles/): records that fit one
    // 76-byte register window pack 4 consecutive rows per lane; longer ones
    // would hold 4 records x several windows of VGPRs, so they take one row
    // per lane (or 2 consecutive rows up to 152 B with NGZ_RTC_LONG=c2).
    int rpl = 4;
    bool consec = true;
    //
    // LDS-staged kernels take rows 64 apart ("r1" by default): a load
    // instruction's 64 lanes then read 64 adjacent records (one contiguous
    // span), where 4 consecutive rows per lane spread it over 4x as many
    // cache lines; T20 at 10^8 records decoded in 2.15 ms (r1) vs 2.55 ms
    // (c4) on the same box (profiles/r1e).
    const char *layout = ngz_knob_str("NGZ_RTC_LAYOUT", nullptr);
    if (!layout && P.lds_waves) layout = ngz_knob_str("NGZ_RTC_LDS_LAYOUT", "r1");
    if (!layout && P.rec_len > 76) layout = ngz_knob_str("NGZ_RTC_LONG", "r1");
    if (layout) {
        if (layout[0] == 'c' || layout[0] == 'r') {
            consec = layout[0] == 'c';
            rpl = atoi(layout + 1);
        }
        if (rpl != 1 && rpl != 2 && rpl != 4) rpl = 4;
    }
    // LDS-staged kernels stage the columns narrower than P.reserved0 bytes (all
    // of them when 0) in LDS; wider columns (64 lanes x 8-16 B = 0.5-1 KB per
    // store instruction already) are stored to HBM directly, so the LDS window
    // holds more rows and more waves fit a CU.  lds_col[f]: the field's column
    // offset factor inside the staged (LDS) row.
    const uint32_t lw0 = P.lds_waves;
    std::vector<uint32_t> lds_col(P.n_fields, 0);
    std::vector<uint8_t> direct(P.n_fields, 0);
    uint32_t staged_rowb = 0;
    for (uint32_t f = 0; f < P.n_fields; ++f) {
        const DevField &d = P.f[f];
        uint32_t same = f;  // pieces of one raw field share a column
        for (uint32_t g = 0; g < f; ++g)
            if (P.f[g].width && P.f[g].col_off == d.col_off) { same = g; break; }
        if (same != f) { lds_col[f] = lds_col[same]; direct[f] = direct[same]; continue; }
        direct[f] = lw0 && P.reserved0 && d.width >= P.reserved0;
        if (!direct[f]) { lds_col[f] = staged_rowb; staged_rowb += d.width; }
    }
    std::string body;
    char b[512];
    auto emit_item = [&](const Item &it, uint32_t wb, int k) {
        const std::string R = "R[" + std::to_string(k) + "]", P = "P[" + std::to_string(k) + "]";
        const bool dir = direct[it.f];
        const uint32_t co = (lw0 && !dir) ? lds_col[it.f] : it.col_off;
        switch (it.type) {
        case 0:
            snprintf(b, sizeof b, "        dec_num<%s>(%s, %s, %uu, %uu, %uu, %uu, %uu, %uu, %uu);\n", dir ? "ColGlb" : "ColT",
                     R.c_str(), P.c_str(), it.off - wb, it.off, it.f, it.len, it.width, it.kind, co);
            break;
        case 1:
            snprintf(b, sizeof b, "        dec_raw<%s>(%s, %s, %uu, %uu, %uu, %uu, %uu, %uu);\n", dir ? "ColGlb" : "ColT",
                     R.c_str(), P.c_str(), it.off + it.j - wb, it.j, it.piece, it.width, co, it.pad_to);
            break;
        case 2:
            snprintf(b, sizeof b, "        check_str(%s, %s, %uu, %uu, %uu, %uu, true);\n", R.c_str(), P.c_str(),
                     it.off - wb, it.off, it.f, it.len);
            break;
        case 3:
            snprintf(b, sizeof b, "        check_str(%s, %s, 0u, %uu, %uu, %uu, false);\n", R.c_str(), P.c_str(), it.off,
                     it.f, it.len);
            break;
        case 4:
            snprintf(b, sizeof b, "        fail_field(%s, %uu, %uu);\n", P.c_str(), it.off, it.f);
            break;
        }
        body += b;
    };
    // per window: the loads of all rows first, then its items
    size_t i = 0;
    while (i < items.size()) {
        size_t e = i + 1;
        while (e < items.size() && item_win[e] == item_win[i]) ++e;
        const int w = item_win[i];
        if (w >= 0) {
            for (int k = 0; k < rpl; ++k) {
                snprintf(b, sizeof b, "        win_load<%u>(R[%d], P[%d], %uu);\n", wins[w].second, k, k, 4 * wins[w].first);
                body += b;
            }
        }
        const uint32_t wb = w >= 0 ? 4 * wins[w].first : 0;
        if (consec) {
            for (size_t t = i; t < e; ++t) {
                const Item &it = items[t];
                const uint32_t co = lw0 ? lds_col[it.f] : it.col_off;
                if (direct[it.f]) {
                    for (int k = 0; k < rpl; ++k) emit_item(it, wb, k);
                } else if (it.type == 0) {
                    snprintf(b, sizeof b, "        dec_num_c<%d, ColT>(R, P, %uu, %uu, %uu, %uu, %uu, %uu, %uu);\n", rpl,
                             it.off - wb, it.off, it.f, it.len, it.width, it.kind, co);
                    body += b;
                } else if (it.type == 1 && it.j == 0 && it.piece == it.len && it.len == it.width && it.width <= 16) {
                    // whole short raw field: packed C-row store
                    snprintf(b, sizeof b, "        dec_raw_c<%d, ColT>(R, P, %uu, %uu, %uu);\n", rpl, it.off - wb, it.width, co);
                    body += b;
                } else {
                    for (int k = 0; k < rpl; ++k) emit_item(it, wb, k);
                }
            }
        } else {
            for (int k = 0; k < rpl; ++k)
                for (size_t t = i; t < e; ++t) emit_item(items[t], wb, k);
        }
        i = e;
    }
    FixedParts out;
    out.rpl = rpl;
    out.consec = consec;
    out.lw = P.lds_waves;
    out.rowb = staged_rowb;
    out.rec_len = P.rec_len;
    out.pass = body;
    const uint32_t lw = P.lds_waves;
    if (lw) {
        // Store step of the LDS-staged kernel: each column's run of the window
        // (LDS_ROWS*width bytes) cut into 1 KB units (64 lanes x 16 B), dealt
        // round robin to the waves; every store instruction is one full wave
        // writing 1 KB of one column.
        const uint32_t rows = NGZ_REG_WINDOW * lw;
        std::vector<std::string> per_wave(lw);
        uint32_t u = 0;
        for (uint32_t f = 0; f < P.n_fields; ++f) {
            const DevField &d = P.f[f];
            if (!d.width || direct[f]) continue;
            // pieces of one raw field share its column: one run per column
            bool seen = false;
            for (uint32_t g = 0; g < f; ++g) seen = seen || (P.f[g].width && P.f[g].col_off == d.col_off);
            if (seen) continue;
            const uint32_t run = rows * d.width;
            for (uint32_t at = 0; at < run; at += 1024, ++u) {
                const uint32_t lanes = std::min<uint32_t>(1024, run - at) / 16;
                snprintf(b, sizeof b,
                         "            lds_flush(blk + (uint64_t)cap * %uu + (uint64_t)W * %uu, %uu, %uu, %uu);\n",
                         d.col_off, run, at, rows * lds_col[f] + at, lanes);
                per_wave[u % lw] += b;
            }
        }
        // NGZ_RTC_EXP=1: no store step (timing experiments only; output invalid)
        if (ngz_knob("NGZ_RTC_EXP", 0) & 1) per_wave.assign(lw, "");
        std::string st;
        st += "    auto store = [&](uint32_t W, uint8_t *blk, uint32_t cap) {\n";
        st += "        const uint32_t q = sgpr(threadIdx.x >> 6);\n";
        for (uint32_t q = 0; q < lw; ++q) {
            st += q ? "        else if (q == " + std::to_string(q) + ") {\n" : "        if (q == 0) {\n";
            st += per_wave[q];
            st += "        }\n";
        }
        st += "    };\n";
        out.store = st;
    }
    return out;
}

// The lambdas of one fixed template's decode: shape, pass and (LDS-staged) store.
std::string fixed_lambdas(const FixedParts &F) {
    const std::string RPL = std::to_string(F.rpl);
    std::string src;
    src += "    auto shape = [](uint32_t) { return RecShape{" + std::to_string(F.rec_len) + "u, 0u, false}; };\n";
    src += "    auto pass = [&](const Pass (&P)[" + RPL + "]) {\n";
    src += "        uint32_t R[" + RPL + "][WIN_DW];\n";
    src += F.pass;
    src += "    };\n";
    src += F.store;
    return src;
}

std::string generate(const DevPlan &P) {
    if (P.has_vlen || staged_rows(P)) return generate_vlen(P);
    const FixedParts F = fixed_parts(P);
    const std::string L = std::to_string(F.rpl) + ", " + (F.consec ? "true" : "false");
    const uint32_t lw = F.lw;
    std::string src;
    src += "// generated by ngz_rtc.cpp for plan " + signature(P) + "\n";
    if (lw) {
        src += "#define NGZ_LDS_WAVES " + std::to_string(lw) + "\n";
        src += "#define NGZ_LDS_ROWB " + std::to_string(F.rowb) + "\n";
    }
    src += cpol_defines() + "#include \"ngz_dev.h\"\nusing namespace ngzdev;\n";
    src += "extern \"C\" __global__ void __launch_bounds__(" + std::to_string(lw ? 64 * lw : 256) +
           ") ngz_tpl(BatchDev B, uint32_t slot) {\n";
    src += "    if (sload(&B.summary->overflow)) return;\n";
    src += "    const SlotRT rt = sload(&B.slots[slot]);\n";
    src += "    const uint32_t c0 = rt.chunk0, nc = rt.nchunks;\n";
    src += "    using ColT = ColSt;\n";
    src += fixed_lambdas(F);
    if (lw) {
        const std::string rows = std::to_string(NGZ_REG_WINDOW * lw);
        src += "    (void)c0; (void)nc;\n";
        src += "    run_lds<" + L + ", " + std::to_string(lw) + ">(B, slot, shape, pass, store, win_seq((rt.total + " + rows +
               " - 1) / " + rows + "));\n}\n";
        return src;
    }
    src += "    if (rt.mode == NGZ_MODE_ROW) run_windows<" + L + ">(B, slot, shape, pass);\n";
    src += "    else run_chunks<" + L + ">(B, c0, c0 + nc, [](uint32_t) { return true; }, shape, pass);\n}\n";
    return src;
}

// One launch for several LDS-staged fixed templates of the same workgroup shape
// (lds_waves): ngz_tplm(B, slots) runs each template's windows in turn, dealt
// XCD-aware over the whole grid (win_seq), each decoded by its own specialised
// body (every field a constant, as in ngz_tpl).
// Against one launch per template, the batch has one ramp and one tail instead
// of one per template (config 3: 8 launches of 1.25e7 records each ran 10-15 %
// below the per-byte rate of one 1e8-record launch).
std::string generate_group(const DevPlan *const *plans, uint32_t n) {
    std::string src;
    src += "// generated by ngz_rtc.cpp: multi-template kernel of " + std::to_string(n) + " plans\n";
    uint32_t lds = 0, lw = plans[0]->lds_waves;
    std::vector<FixedParts> parts;
    for (uint32_t k = 0; k < n; ++k) {
        parts.push_back(fixed_parts(*plans[k]));
        lds = std::max<uint32_t>(lds, NGZ_REG_WINDOW * parts.back().lw * parts.back().rowb);
    }
    src += "#define NGZ_LDS_BYTES " + std::to_string(std::max<uint32_t>(lds, 16)) + "\n";
    src += cpol_defines() + "#include \"ngz_dev.h\"\nusing namespace ngzdev;\n";
    for (uint32_t k = 0; k < n; ++k) {
        const FixedParts &F = parts[k];
        const std::string L = std::to_string(F.rpl) + ", " + (F.consec ? "true" : "false");
        src += "namespace t" + std::to_string(k) + " {  // " + signature(*plans[k]) + "\n";
        src += "__device__ __forceinline__ void run(const BatchDev &B, uint32_t slot, const WinSeq ws) {\n";
        src += "    using ColT = ColLds<" + std::to_string(NGZ_REG_WINDOW * F.lw) + ">;\n";
        src += fixed_lambdas(F);
        src += "    run_lds<" + L + ", " + std::to_string(F.lw) + ">(B, slot, shape, pass, store, ws);\n}\n}\n";
    }
    src += "struct NgzSlots { uint32_t s[" + std::to_string(NGZ_RTC_GROUP_MAX) + "]; };\n";
    src += "extern \"C\" __global__ void __launch_bounds__(" + std::to_string(64 * lw) +
           ") ngz_tplm(BatchDev B, NgzSlots S) {\n";
    src += "    if (sload(&B.summary->overflow)) return;\n";
    // every template's windows dealt over the whole grid as its own kernel would (win_seq: an
    // eighth per XCD), one template after the other: each XCD takes an eighth of every template,
    // so per-window costs that differ by template (40- to 153-byte records) stay balanced across
    // the XCDs, and a workgroup goes on to the next template's windows without a kernel boundary
    const std::string rows = std::to_string(NGZ_REG_WINDOW * lw);
    src += "    uint32_t nw;\n";
    for (uint32_t k = 0; k < n; ++k) {
        const std::string K = std::to_string(k);
        src += "    nw = (sload(&B.slots[S.s[" + K + "]]).total + " + rows + " - 1) / " + rows + ";\n";
        src += "    if (nw) t" + K + "::run(B, S.s[" + K + "], win_seq(nw));\n";
    }
    src += "}\n";
    return src;
}

// Templates with variable-length fields (IPFIX length 65535, RFC 7011 s7):
// records are found by the framing walk (ngz_vlen_walk, per-row record
// offsets) and decoded one record per lane in row mode.  The fields between
// two variable-length fields form a segment whose offsets relative to the
// segment start are constants, so each segment is decoded like a small fixed
// template: statically planned register windows at the lane's segment start
// (16-byte aligned loads re-aligned per lane, as for unaligned fixed records),
// constant extraction offsets.  A variable-length field reads its u8 / 255 +
// 3-byte length (generator.rs:1775-1793) from the window, stores
// {u64 batch offset, u32 length, 0}, checks UTF-8 for strings (no NUL
// truncation, generator.rs:1635-1672) and moves the lane's segment start past
// its value.  Replaces the generic kernel's field-table walk with run-time
// register indexing for these templates.
// Fixed templates decoded by the staged-row kernel shape (see ngz_host.cpp: NetFlow v9 templates of
// up to NGZ_VSTAGE_REC_MAX-byte records): row-mode batches copy each 64-row group's records into LDS,
// chunk-mode batches (sets of 64+ records on average) read them through the chunk's resource
bool staged_rows(const DevPlan &P) {
    return !P.has_vlen && P.rpl && !P.lds_waves && P.proto == 9 && P.rec_len <= NGZ_VSTAGE_REC_MAX;
}

// Staged-row kernels of fixed records (NetFlow v9, staged_rows): the pass of a row-mode group keeps
// every decoded cell in registers, then, once the wave's reads of its LDS record image are done,
// writes the 64 rows' cells into that image column-major (column c at 64 * col_off, its rows
// contiguous) and stores the image to the columns 16 bytes per lane: piece p of the image is the
// 16-byte piece p - 4 col_off of column c's run for the group (piece_table).  A wave's 64 rows
// then go out in ceil(row_bytes / 16) store instructions of 64 x 16 B instead of one narrow store
// per field (1-8 B per lane: the NFv9 313 launch issued 44 store instructions per group, 215 B
// each, and waited to issue 49 % of its wave cycles, profiles/r6h/cfg4/pmc_dispatch.txt).  The
// group's last rows past the slot's total are padding rows of the column capacity (a multiple of
// 256), so whole pieces are stored.  Chunk-mode batches keep the per-field stores (a chunk's rows
// end inside a group).  Empty when the plan does not qualify: rows over 160 bytes (the image holds
// 64 rows of 160 B), or a field too wide for registers.
std::string piece_table(const DevPlan &P) {
    std::string t = "__constant__ uint32_t ngz_pt[" + std::to_string(4 * P.row_bytes) + "] = {";
    char b[32];
    for (uint32_t f = 0, n = 0; f < P.n_fields; ++f) {
        const DevField &d = P.f[f];
        if (!d.width) continue;
        for (uint32_t k = 0; k < 4 * d.width; ++k, ++n) {
            snprintf(b, sizeof b, "%s%uu", n ? "," : "", d.col_off | (d.width << 8) | (k << 16));
            t += b;
        }
    }
    return t + "};\n";
}

std::string staged_row_body(const DevPlan &P, const std::vector<Item> &items) {
    if (P.has_vlen || P.row_bytes == 0 || P.row_bytes > 160 || 64 * P.row_bytes > NGZ_VSTAGE_IMAGE) return {};
    for (uint32_t f = 0, co = 0; f < P.n_fields; ++f) {  // columns back to back in field order
        if (P.f[f].width && P.f[f].col_off != co) return {};
        co += P.f[f].width;
    }
    for (const Item &it : items)
        if (it.type == 3 || it.type == 5 || (it.type == 1 && (it.j || it.piece != it.len || it.width > 32 || it.pad_to != it.width)))
            return {};
    std::string s;
    char b[1024];
    s += "        const Pass &P0 = P[0];\n";
    s += "        Pass Q = P0;\n";
    s += "        const uint32_t seg = 0;\n";
    s += "        (void)seg;\n";
    // windows: greedy in record order, as generate_vlen plans them
    std::vector<std::pair<uint32_t, uint32_t>> wins;
    std::vector<int> item_win(items.size(), -1);
    for (size_t i = 0; i < items.size(); ++i) {
        const Item &it = items[i];
        if (it.type == 4) continue;
        if (wins.empty() || it.d0 < wins.back().first || it.d1 >= wins.back().first + kWinDw) wins.push_back({it.d0, 1});
        auto &w = wins.back();
        w.second = std::max(w.second, it.d1 - w.first + 1);
        item_win[i] = (int)wins.size() - 1;
    }
    std::string stage;  // the cells into the LDS image, after every read of it
    int cur = -1;
    for (size_t i = 0; i < items.size(); ++i) {
        const Item &it = items[i];
        const int w = item_win[i];
        if (w >= 0 && w != cur) {
            snprintf(b, sizeof b, "        win_load_v<%u>(R[0], Q, %uu);\n", wins[w].second, 4 * wins[w].first);
            s += b;
            cur = w;
        }
        const uint32_t wb = w >= 0 ? 4 * wins[w].first : 0;
        const uint32_t o = it.off - wb, at = 64 * it.col_off;
        switch (it.type) {
        case 0:
            snprintf(b, sizeof b, "        const uint64_t v%u = num_value(R[0], P0, %uu, %uu, %uu, %uu, %uu);\n", it.f, o,
                     it.off, it.f, it.len, it.kind);
            s += b;
            if (it.width == 1) snprintf(b, sizeof b, "            st[%uu + lane] = (uint8_t)v%u;\n", at, it.f);
            else if (it.width == 2) snprintf(b, sizeof b, "            *(uint16_t *)&st[%uu + 2 * lane] = (uint16_t)v%u;\n", at, it.f);
            else if (it.width == 4) snprintf(b, sizeof b, "            *(uint32_t *)&st[%uu + 4 * lane] = (uint32_t)v%u;\n", at, it.f);
            else snprintf(b, sizeof b, "            *(uint64_t *)&st[%uu + 8 * lane] = v%u;\n", at, it.f);
            stage += b;
            break;
        case 1: {  // raw cell: len bytes, width == len (<= 32), into ceil(width / 4) dwords
            const uint32_t nd = (it.width + 3) / 4;
            for (uint32_t m = 0; m < nd; ++m) {
                if (4 * m + 4 <= it.len) {
                    snprintf(b, sizeof b, "        const uint32_t c%u_%u = rdw(R[0], %uu);\n", it.f, m, o + 4 * m);
                } else {
                    std::string e = "0u";
                    for (uint32_t q = 4 * m; q < std::min(4 * m + 4, it.len); ++q)
                        e += " | (rbyte(R[0], " + std::to_string(o + q) + "u) << " + std::to_string(8 * (q - 4 * m)) + ")";
                    snprintf(b, sizeof b, "        const uint32_t c%u_%u = %s;\n", it.f, m, e.c_str());
                }
                s += b;
            }
            if ((it.width & 3) == 0) {
                for (uint32_t m = 0; m < nd; ++m) {
                    snprintf(b, sizeof b, "            *(uint32_t *)&st[%uu + %uu * lane + %uu] = c%u_%u;\n", at, it.width,
                             4 * m, it.f, m);
                    stage += b;
                }
            } else {
                for (uint32_t q = 0; q < it.width; ++q) {
                    snprintf(b, sizeof b, "            st[%uu + %uu * lane + %uu] = (uint8_t)(c%u_%u >> %u);\n", at,
                             it.width, q, it.f, q / 4, 8 * (q % 4));
                    stage += b;
                }
            }
            break;
        }
        case 2:
            snprintf(b, sizeof b, "        check_str(R[0], P0, %uu, %uu, %uu, %uu, true);\n", o, it.off, it.f, it.len);
            s += b;
            break;
        case 4:
            snprintf(b, sizeof b, "        fail_field(P0, %uu, %uu);\n", it.off, it.f);
            s += b;
            break;
        }
    }
    s += "        {  // stage the group's cells in the wave's image (every lane's reads of it are done), then store\n";
    s += "            const uint32_t lane = threadIdx.x & 63;\n";
    s += "            uint8_t *st = (uint8_t *)&ngz_vstage[(threadIdx.x >> 6) * kVStageDw];\n";
    s += "            __builtin_amdgcn_fence(__ATOMIC_RELEASE, \"wavefront\");\n"
         "            __builtin_amdgcn_wave_barrier();\n"
         "            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, \"wavefront\");\n";
    s += stage;
    s += "            __builtin_amdgcn_fence(__ATOMIC_RELEASE, \"wavefront\");\n"
         "            __builtin_amdgcn_wave_barrier();\n"
         "            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, \"wavefront\");\n";
    snprintf(b, sizeof b,
             "            for (uint32_t p = lane; p < %uu; p += 64) {\n"
             "                const uint32_t e = ngz_pt[p];\n"
             "                const v4u x = *(const v4u *)&st[16 * p];\n"
             "                uint8_t *d = P0.blk + (uint64_t)P0.cap * (e & 0xFFu) + (uint64_t)P0.prow * ((e >> 8) & 0xFFu) +\n"
             "                             16u * (e >> 16);\n"
             "                __builtin_nontemporal_store(x, (v4u *)d);\n"
             "            }\n"
             "            __builtin_amdgcn_fence(__ATOMIC_RELEASE, \"wavefront\");\n"
             "            __builtin_amdgcn_wave_barrier();\n"
             "            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, \"wavefront\");\n"
             "        }\n",
             4 * P.row_bytes);
    s += b;
    return s;
}

std::string generate_vlen(const DevPlan &P) {
    struct Seg {
        std::vector<Item> items;   // fixed fields, offsets relative to the segment start
        int vf = -1;               // variable-length field ending the segment
        uint32_t vpos = 0;         // its length prefix, relative to the segment start
    };
    std::vector<Seg> segs(1);
    uint32_t so = 0;
    for (uint32_t f = 0; f < P.n_fields; ++f) {
        const DevField &d = P.f[f];
        Seg &sg = segs.back();
        Item it{};
        it.f = f;
        it.off = so;
        it.len = d.len;
        it.width = d.width;
        it.kind = d.kind;
        it.col_off = d.col_off;
        switch (d.kind) {
        case NGZ_K_VLEN:
            sg.vf = (int)f;
            sg.vpos = so;
            segs.emplace_back();
            so = 0;
            continue;
        case NGZ_K_FAIL:
            it.type = 4;
            sg.items.push_back(it);
            break;
        case NGZ_K_UINT: case NGZ_K_SCOPE32: case NGZ_K_TCPFLAGS: case NGZ_K_SINT:
        case NGZ_K_BOOL: case NGZ_K_DTMS: case NGZ_K_DTFRAC: {
            uint32_t L = d.len;
            if (d.kind == NGZ_K_DTMS || d.kind == NGZ_K_DTFRAC) L = 8;
            if (d.kind == NGZ_K_BOOL) L = 1;
            if (L == 0) L = 1;
            it.type = 0;
            it.d0 = so >> 2;
            it.d1 = (so + L - 1) >> 2;
            sg.items.push_back(it);
            break;
        }
        case NGZ_K_STR: case NGZ_K_BYTES: case NGZ_K_U256: {
            if (d.kind == NGZ_K_STR) {
                Item c = it;
                c.type = d.len <= 64 ? 2 : 3;
                c.d0 = so >> 2;
                c.d1 = d.len ? (so + d.len - 1) >> 2 : c.d0;
                sg.items.push_back(c);
            }
            for (uint32_t j = 0;; j += 64) {
                Item r = it;
                r.type = 1;
                r.j = j;
                r.piece = std::min<uint32_t>(64, d.len - j);
                const bool last = j + 64 >= d.len;
                r.pad_to = last ? d.width : 0;
                r.d0 = (so + j) >> 2;
                r.d1 = r.piece ? (so + j + r.piece - 1) >> 2 : r.d0;
                sg.items.push_back(r);
                if (last) break;
            }
            break;
        }
        default:
            break;
        }
        so += d.len;
    }
    // NGZ_RTC_EXP (experiment build only; timing attribution, output invalid): bit 1 no UTF-8
    // checks of variable-length strings, bit 3 an empty decode (the staging copy alone)
    const int64_t vexp = ngz_knob("NGZ_RTC_EXP", 0);
    std::string body;
    char b[640];
    body += "        const Pass &P0 = P[0];\n";
    body += "        Pass Q = P0;                              // window loads relative to the segment start\n";
    body += "        const uint32_t rel0 = P0.rbase + P0.sh;   // record start, relative to the resource\n";
    body += "        uint32_t seg = 0;                         // per lane: record offset of the segment\n";
    body += "        (void)rel0; (void)seg;\n";
    for (size_t si = 0; si < segs.size(); ++si) {
        Seg &sg = segs[si];
        // the length prefix of the closing vlen field is read from the segment's windows too
        std::vector<Item> items = sg.items;
        if (sg.vf >= 0) {
            Item v{};
            v.type = 5;
            v.f = (uint32_t)sg.vf;
            v.off = sg.vpos;
            v.d0 = sg.vpos >> 2;
            v.d1 = (sg.vpos + 3) >> 2;
            items.push_back(v);
        }
        // windows: greedy in segment order
        std::vector<std::pair<uint32_t, uint32_t>> wins;
        std::vector<int> item_win(items.size(), -1);
        for (size_t i = 0; i < items.size(); ++i) {
            const Item &it = items[i];
            if (it.type == 3 || it.type == 4) continue;
            if (wins.empty() || it.d0 < wins.back().first || it.d1 >= wins.back().first + kWinDw) wins.push_back({it.d0, 1});
            auto &w = wins.back();
            w.second = std::max(w.second, it.d1 - w.first + 1);
            item_win[i] = (int)wins.size() - 1;
        }
        int cur = -1;
        for (size_t i = 0; i < items.size(); ++i) {
            const Item &it = items[i];
            const int w = item_win[i];
            if (w >= 0 && w != cur) {
                snprintf(b, sizeof b, "        win_load_v<%u>(R[0], Q, %uu);\n", wins[w].second, 4 * wins[w].first);
                body += b;
                cur = w;
            }
            const uint32_t wb = w >= 0 ? 4 * wins[w].first : 0;
            switch (it.type) {
            case 0:
                snprintf(b, sizeof b, "        dec_num(R[0], P0, %uu, seg + %uu, %uu, %uu, %uu, %uu, %uu);\n", it.off - wb,
                         it.off, it.f, it.len, it.width, it.kind, it.col_off);
                break;
            case 1:
                snprintf(b, sizeof b, "        dec_raw(R[0], P0, %uu, %uu, %uu, %uu, %uu, %uu);\n", it.off + it.j - wb, it.j,
                         it.piece, it.width, it.col_off, it.pad_to);
                break;
            case 2:
                snprintf(b, sizeof b, "        check_str(R[0], P0, %uu, seg + %uu, %uu, %uu, true);\n", it.off - wb, it.off,
                         it.f, it.len);
                break;
            case 3:
                snprintf(b, sizeof b,
                         "        if (P0.valid && !utf8_valid_v(P0, rel0 + seg + %uu, %uu, true))"
                         " rec_error(P0, seg + %uu, E_REC_UTF8, %uu);\n",
                         it.off, it.len, it.off, it.f);
                break;
            case 4:
                snprintf(b, sizeof b, "        fail_field(P0, seg + %uu, %uu);\n", it.off, it.f);
                break;
            case 5: {
                const DevField &d = P.f[it.f];
                const std::string F = std::to_string(it.f);
                body += "        {  // variable-length field " + F + "\n";
                snprintf(b, sizeof b,
                         "            uint32_t L = rbyte(R[0], %uu), hdr = 1;\n"
                         "            if (L == 255) { L = (uint32_t)rbe(R[0], %uu, 3); hdr = 4; }\n"
                         "            const uint32_t data = seg + %uu + hdr;\n"
                         "            if (P0.valid) {\n"
                         "                const uint64_t at = P0.rabs + data;\n"
                         "                ColSt(P0, %uu, 16).b128(P0.lrow * 16, (uint32_t)at, (uint32_t)(at >> 32), L, 0);\n",
                         it.off - wb, it.off + 1 - wb, it.off, d.col_off);
                body += b;
                if ((d.flags & 0x80) && !(vexp & 2))  // string: every byte UTF-8 checked
                    body += "                if (!utf8_valid_v(P0, rel0 + data, L, false))\n"
                            "                    rec_error(P0, data, E_REC_UTF8, " + F + "u, L);\n";
                body += "            }\n"
                        "            seg = data + L;\n"
                        "            Q.rbase = (rel0 + seg) & ~3u;\n"
                        "            Q.sh = (rel0 + seg) & 3u;\n"
                        "            Q.any_sh = __builtin_amdgcn_ballot_w64(Q.sh != 0) != 0;\n"
                        "        }\n";
                cur = -1;  // the next segment needs its own windows
                break;
            }
            }
            if (it.type != 5) body += b;
        }
    }
    const std::string sbody = P.has_vlen ? std::string() : staged_row_body(P, segs[0].items);
    std::string src;
    src += "// generated by ngz_rtc.cpp for plan " + signature(P) + "\n";
    src += cpol_defines() + "#define NGZ_VSTAGE 1\n#include \"ngz_dev.h\"\nusing namespace ngzdev;\n";
    if (!sbody.empty()) src += piece_table(P);
    src += "extern \"C\" __global__ void __launch_bounds__(256) ngz_tpl(BatchDev B, uint32_t slot) {\n";
    src += "    if (sload(&B.summary->overflow)) return;\n";
    src += "    auto pass = [&](const Pass (&P)[1]) {\n";
    src += "        uint32_t R[1][WIN_DW];\n";
    src += (vexp & 8) ? std::string("        (void)P; (void)R;\n") : body;
    src += "    };\n";
    if (!sbody.empty()) {
        src += "    auto pass_rows = [&](const Pass (&P)[1]) {\n";
        src += "        uint32_t R[1][WIN_DW];\n";
        src += sbody;
        src += "    };\n";
    }
    if (P.has_vlen) {
        src += "    run_windows_staged(B, slot, pass);\n}\n";
    } else if (!sbody.empty()) {
        snprintf(b, sizeof b,
                 "    const SlotRT rt = sload(&B.slots[slot]);\n"
                 "    if (rt.mode == NGZ_MODE_ROW) {\n"
                 "        run_windows_staged(B, slot, pass_rows);\n"
                 "    } else {\n"
                 "        auto want = [&](uint32_t s) { return s == slot; };\n"
                 "        auto shape = [](uint32_t) { return RecShape{%uu, 0u, false}; };\n"
                 "        run_chunks<1, false>(B, rt.chunk0, rt.chunk0 + rt.nchunks, want, shape, pass);\n"
                 "    }\n}\n",
                 P.rec_len);
        src += b;
    } else {
        snprintf(b, sizeof b,
                 "    const SlotRT rt = sload(&B.slots[slot]);\n"
                 "    if (rt.mode == NGZ_MODE_ROW) {\n"
                 "        run_windows_staged(B, slot, pass);\n"
                 "    } else {\n"
                 "        auto want = [&](uint32_t s) { return s == slot; };\n"
                 "        auto shape = [](uint32_t) { return RecShape{%uu, 0u, false}; };\n"
                 "        run_chunks<1, false>(B, rt.chunk0, rt.chunk0 + rt.nchunks, want, shape, pass);\n"
                 "    }\n}\n",
                 P.rec_len);
        src += b;
    }
    return src;
}

struct Entry {
    std::atomic<int> state{0};  // 0 new, 1 compiling, 2 ready, 3 failed
    hipModule_t mod = nullptr;
    hipFunction_t fn = nullptr;
};

std::mutex g_mu;  // the map only; never held across a compile
std::map<std::pair<int, std::string>, std::unique_ptr<Entry>> g_cache;

// Background compiles never outlive the runtime they compile and load modules
// with.  They are joined by an exit handler, and exit handlers run in the
// reverse order of their registration -- static destructors of a library
// included, registered when the library is loaded.  The compiler hiprtc drives
// (libamd_comgr, LLVM) is not linked in: hiprtc dlopens it on its first
// program, i.e. on the first worker thread, after a handler registered when
// that worker started.  Exit then ran comgr's / LLVM's static destructors
// first, under a compile still inside them, and the join waited on a thread
// that could not finish (the exit hang of a dist rank in r2).  So the handler
// is registered once hiprtc and comgr are loaded and initialised
// (prime_rtc_runtime): every destructor they register comes before it and
// runs after the join.
//
// That ordering is not enough on its own: comgr / LLVM also construct
// function-local statics during a compile, on the worker, and those register
// their destructors after the handler, so exit runs them first.  A dist rank
// that exited with compiles in flight still hung in r3.  The complete rule is
// that no compile is in flight when the exit handlers start.  The pool keeps
// the entries queued or compiling: ngz_ctx_destroy waits for those of every
// entry its context started or waits on (ngz_rtc_join), so a C / Rust
// host that destroys its contexts (the codec's drop is synchronous,
// codec.rs:68-82) has nothing in flight when it returns from main;
// ngz_rtc_drain waits for every queued compile (netgauze_amd._lib registers it with
// Python's atexit, which runs before any C exit handler).
//
// Compiles run on a bounded pool (kMaxCompilers threads draining one queue), not one thread
// per template: a peer announcing hundreds of templates at once (or the differential fuzz
// corpus, tests/test_gpu_fuzz.py: ~600 distinct layouts) used to start hundreds of
// concurrent hiprtc compiles, each with its own LLVM context.  A pool thread ends when the
// queue is empty; the next submit after that reaps the finished threads.
void build(Entry *e, int device, const std::string &src, const std::string &sig, const char *kname);

struct Workers {
    static constexpr size_t kMaxCompilers = 4;
    struct Job {
        Entry *e;
        int device;
        std::string src, sig;
        const char *kname;
    };
    std::mutex mu;
    std::condition_variable cv;            // a job finished or a thread ended
    std::deque<Job> q;                     // not started yet
    std::vector<std::thread> th;           // pool threads, running or ended and not yet joined
    size_t running = 0;                    // threads still draining the queue
    std::multiset<const void *> pending;   // entries queued or compiling
    void submit(Job j) {
        std::vector<std::thread> ended;
        {
            std::lock_guard<std::mutex> lk(mu);
            if (running == 0) ended.swap(th);  // every earlier thread left its loop
            pending.insert(j.e);
            q.push_back(std::move(j));
            if (running < kMaxCompilers) {
                ++running;
                th.emplace_back([this] { loop(); });
            }
        }
        for (auto &t : ended)
            if (t.joinable()) t.join();
    }
    void loop() {
        pthread_setname_np(pthread_self(), "ngz-rtc");  // visible in /proc/<pid>/task/*/comm
        std::unique_lock<std::mutex> lk(mu);
        while (!q.empty()) {
            Job j = std::move(q.front());
            q.pop_front();
            lk.unlock();
            build(j.e, j.device, j.src, j.sig, j.kname);
            lk.lock();
            pending.erase(pending.find(j.e));
            cv.notify_all();
        }
        --running;
        cv.notify_all();
    }
    // wait until none of the given entries is queued or compiling; returns how many were
    int join(const void *const *entries, size_t n) {
        std::unique_lock<std::mutex> lk(mu);
        int k = 0;
        for (size_t i = 0; i < n; ++i) k += pending.count(entries[i]) ? 1 : 0;
        cv.wait(lk, [&] {
            for (size_t i = 0; i < n; ++i)
                if (pending.count(entries[i])) return false;
            return true;
        });
        return k;
    }
    // wait for the queue to drain and every pool thread to end; returns the compiles waited for
    int join_all() {
        std::vector<std::thread> v;
        int k;
        {
            std::unique_lock<std::mutex> lk(mu);
            k = (int)pending.size();
            cv.wait(lk, [&] { return q.empty() && running == 0; });
            v.swap(th);
        }
        for (auto &t : v)
            if (t.joinable()) t.join();
        return k;
    }
    // exit: compiles not started are dropped (their entries fail: nobody decodes any more)
    void cancel_queued() {
        std::lock_guard<std::mutex> lk(mu);
        for (Job &j : q) {
            j.e->state.store(3, std::memory_order_release);
            pending.erase(pending.find(j.e));
        }
        q.clear();
        cv.notify_all();
    }
    ~Workers() {
        cancel_queued();
        join_all();
    }
} g_workers;

void join_workers_at_exit() {
    g_workers.cancel_queued();
    g_workers.join_all();
}

// Loads comgr and runs hiprtc's lazy initialisation on the calling thread (one
// program created and destroyed, nothing compiled), so that their exit-time
// destructors are registered before join_workers_at_exit.
void prime_rtc_runtime() {
    dlopen("libamd_comgr.so.3", RTLD_NOW | RTLD_GLOBAL);  // kept loaded; hiprtc's own dlopen finds it
    hiprtcProgram prog;
    if (hiprtcCreateProgram(&prog, "extern \"C\" __global__ void ngz_prime() {}\n", "ngz_prime.hip", 0, nullptr,
                            nullptr) == HIPRTC_SUCCESS)
        hiprtcDestroyProgram(&prog);
}

Entry *entry_for(int device, const std::string &sig) {
    std::lock_guard<std::mutex> lk(g_mu);
    std::unique_ptr<Entry> &e = g_cache[{device, sig}];
    if (!e) e.reset(new Entry());
    return e.get();
}

bool compile(const std::string &src, std::vector<char> &code, std::string &log) {
    hiprtcProgram prog;
    // hiprtc supplies stdint.h but not stddef.h (flow_decode.h only needs size_t)
    static const char kStddef[] = "#pragma once\ntypedef __SIZE_TYPE__ size_t;\n";
    const char *hdrs[] = {kSrcFlowDecode, kSrcInternal, kSrcDev, kStddef};
    const char *names[] = {"ngz/flow_decode.h", "ngz_internal.h", "ngz_dev.h", "stddef.h"};
    if (hiprtcCreateProgram(&prog, src.c_str(), "ngz_tpl.hip", 4, hdrs, names) != HIPRTC_SUCCESS) return false;
    const char *opts[] = {"--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off"};
    const hiprtcResult rc = hiprtcCompileProgram(prog, 4, opts);
    size_t ls = 0;
    hiprtcGetProgramLogSize(prog, &ls);
    if (ls > 1) {
        log.resize(ls);
        hiprtcGetProgramLog(prog, &log[0]);
    }
    bool ok = rc == HIPRTC_SUCCESS;
    if (ok) {
        size_t cs = 0;
        ok = hiprtcGetCodeSize(prog, &cs) == HIPRTC_SUCCESS && cs > 0;
        if (ok) {
            code.resize(cs);
            ok = hiprtcGetCode(prog, code.data()) == HIPRTC_SUCCESS;
        }
    }
    hiprtcDestroyProgram(&prog);
    return ok;
}



// Compile + load one entry (the caller won the 0 -> 1 transition).
void build(Entry *e, int device, const std::string &src, const std::string &sig, const char *kname) {
    std::vector<char> code;
    std::string log;
    if (ngz_debug_level() >= 2) fprintf(stderr, "[ngz rtc] source:\n%s\n", src.c_str());
    if (!compile(src, code, log)) {
        fprintf(stderr, "[ngz rtc] compile failed for %s:\n%s\n", sig.c_str(), log.c_str());
        e->state.store(3, std::memory_order_release);
        return;
    }
    if (hipSetDevice(device) != hipSuccess || hipModuleLoadData(&e->mod, code.data()) != hipSuccess ||
        hipModuleGetFunction(&e->fn, e->mod, kname) != hipSuccess) {
        fprintf(stderr, "[ngz rtc] module load failed for %s\n", sig.c_str());
        e->fn = nullptr;
        e->state.store(3, std::memory_order_release);
        return;
    }
    e->state.store(2, std::memory_order_release);
}

// A cache entry's kernel, compiled from gen() (kernel `kname`) on first use:
// synchronously (waiting for another thread's compile of it if needed), or in
// the background (ngz_rtc_poll).
template <class Gen>
void *kernel_sync(int device, const std::string &sig, Gen &&gen, const char *kname) {
    Entry *e = entry_for(device, sig);
    int st = 0;
    if (e->state.compare_exchange_strong(st, 1)) {
        build(e, device, gen(), sig, kname);
    } else {
        while ((st = e->state.load(std::memory_order_acquire)) == 1)  // another thread compiles it
            std::this_thread::sleep_for(std::chrono::milliseconds(1));
    }
    return e->state.load(std::memory_order_acquire) == 2 ? (void *)e->fn : nullptr;
}

template <class Gen>
int kernel_async(int device, const std::string &sig, Gen &&gen, const char *kname, void **fn, void **entry) {
    Entry *e = entry_for(device, sig);
    *entry = e;
    int st = 0;
    if (e->state.compare_exchange_strong(st, 1)) {
        std::string src = gen();  // the plans' field tables are the caller's: read them now
        static std::once_flag once;
        std::call_once(once, [] {
            prime_rtc_runtime();
            std::atexit(join_workers_at_exit);
        });
        g_workers.submit(Workers::Job{e, device, std::move(src), sig, kname});
        return 0;
    }
    if (st == 2) {
        *fn = (void *)e->fn;
        return 1;
    }
    return st == 3 ? -1 : 0;
}

std::string group_signature(const DevPlan *const *plans, uint32_t n) {
    std::string s = "G";
    for (uint32_t k = 0; k < n; ++k) s += "|" + signature(*plans[k]);
    return s;
}

}  // namespace

// Specialised kernel for a plan on `device`, compiled on first use and cached,
// waiting for it if needed; nullptr when compilation failed (the caller falls
// back to the generic kernel).
void *ngz_rtc_kernel(int device, const DevPlan &P) {
    return kernel_sync(device, signature(P), [&] { return generate(P); }, "ngz_tpl");
}

// Asynchronous form: returns 1 (ready, *fn set), 0 (compiling in the
// background; poll *entry with ngz_rtc_poll) or -1 (failed).
int ngz_rtc_kernel_async(int device, const DevPlan &P, void **fn, void **entry) {
    return kernel_async(device, signature(P), [&] { return generate(P); }, "ngz_tpl", fn, entry);
}

// The multi-template kernel of n (2..NGZ_RTC_GROUP_MAX) LDS-staged fixed
// plans of one lds_waves (generate_group), in both forms.
void *ngz_rtc_group(int device, const DevPlan *const *plans, uint32_t n) {
    return kernel_sync(device, group_signature(plans, n), [&] { return generate_group(plans, n); }, "ngz_tplm");
}

int ngz_rtc_group_async(int device, const DevPlan *const *plans, uint32_t n, void **fn, void **entry) {
    return kernel_async(device, group_signature(plans, n), [&] { return generate_group(plans, n); }, "ngz_tplm", fn,
                        entry);
}

extern "C" int ngz_rtc_drain(void) {
    // workers started while this runs (another host thread decoding) are joined too
    int n = 0;
    for (int k; (k = g_workers.join_all()) > 0;) n += k;
    return n;
}

// Join the background compiles of these cache entries (whichever context
// started them); returns how many were still registered.
int ngz_rtc_join(void *const *entries, size_t n) { return n ? g_workers.join(entries, n) : 0; }

int ngz_rtc_poll(void *entry, void **fn) {
    Entry *e = (Entry *)entry;
    const int st = e->state.load(std::memory_order_acquire);
    if (st == 2) {
        *fn = (void *)e->fn;
        return 1;
    }
    return st == 3 ? -1 : 0;
}

// The generated source for a plan (introspection / tests).
std::string ngz_rtc_source(const DevPlan &P) { return generate(P); }

// Launch a specialised kernel over one slot's chunks.
int ngz_rtc_launch(void *fn, const BatchDev *B, uint32_t slot, uint32_t grid, uint32_t block, hipStream_t st) {
    BatchDev b = *B;
    uint32_t s = slot;
    void *args[] = {&b, &s};
    return hipModuleLaunchKernel((hipFunction_t)fn, grid, 1, 1, block, 1, 1, 0, st, args, nullptr) == hipSuccess ? 0 : -1;
}

// Launch a multi-template kernel over the slots (the templates' order of the group).
int ngz_rtc_launch_group(void *fn, const BatchDev *B, const uint32_t *slots, uint32_t n, uint32_t grid, uint32_t block,
                         hipStream_t st) {
    if (n > NGZ_RTC_GROUP_MAX) return -1;
    BatchDev b = *B;
    struct {
        uint32_t s[NGZ_RTC_GROUP_MAX];
    } S{};
    for (uint32_t k = 0; k < n; ++k) S.s[k] = slots[k];
    void *args[] = {&b, &S};
    return hipModuleLaunchKernel((hipFunction_t)fn, grid, 1, 1, block, 1, 1, 0, st, args, nullptr) == hipSuccess ? 0 : -1;
}

// The generated multi-template source (introspection / tests).
std::string ngz_rtc_group_source(const DevPlan *const *plans, uint32_t n) { return generate_group(plans, n); }

// Compile a generated source without loading it (no device needed): 0 ok, -1 failed.
int ngz_rtc_compile_source(const std::string &src, std::string *log_out) {
    std::vector<char> code;
    std::string log;
    const bool ok = compile(src, code, log);
    if (log_out) *log_out = log;
    return ok ? 0 : -1;
}

// Generate and compile without loading (no device needed): 0 ok, -1 failed.
int ngz_rtc_compile_only(const DevPlan &P, std::string *log_out) {
    std::vector<char> code;
    std::string log;
    const bool ok = compile(generate(P), code, log);
    if (log_out) *log_out = log;
    return ok ? 0 : -1;
}
