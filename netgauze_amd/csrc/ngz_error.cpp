// ngz_dgram_error: the structured form of a datagram's FlowInfoCodecDecoderError.
//
// The library renders every error as the reference's serde text
// (ngz_dgram_error_json).  This file reads that text back into an ngz_error:
// the chain of enum tags from the outside in gives the layer, the innermost
// variant gives the kind and its fields.  One source of truth: the struct can
// never disagree with the JSON.  IE identity comes from the template (record
// errors: field index of the datagram's error key) or from the specifier in
// the error (template errors).
//
// Reference error enums (crates/flow-pkt/src/wire/deserializer/{ipfix,netflow}.rs,
// codec.rs:44-66, crates/parse-utils/src/error.rs:21-75, generated
// FieldParsingError, generator.rs:1423-1437).
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "ngz/flow_decode.h"
#include "ngz_host.h"

using namespace ngzh;

namespace {

// Minimal reader of the serde shapes the library emits: nested objects,
// arrays, strings, unsigned numbers.
struct JVal {
    enum T { OBJ, ARR, STR, NUM, OTHER } t = OTHER;
    std::vector<std::pair<std::string, JVal>> obj;
    std::vector<JVal> arr;
    std::string str;
    uint64_t num = 0;
    const JVal *get(const char *k) const {
        for (const auto &kv : obj)
            if (kv.first == k) return &kv.second;
        return nullptr;
    }
    uint64_t u(const char *k, uint64_t dflt = 0) const {
        const JVal *v = get(k);
        return v && v->t == NUM ? v->num : dflt;
    }
};

struct JParse {
    const char *p, *e;
    void ws() { while (p < e && (*p == ' ' || *p == '\n' || *p == '\t' || *p == '\r')) ++p; }
    bool str(std::string &out) {
        if (p >= e || *p != '"') return false;
        ++p;
        while (p < e && *p != '"') {
            if (*p == '\\' && p + 1 < e) {
                ++p;
                if (*p == 'u' && p + 4 < e) { out += '?'; p += 5; continue; }
                out += *p == 'n' ? '\n' : *p == 't' ? '\t' : *p;
                ++p;
                continue;
            }
            out += *p++;
        }
        if (p >= e) return false;
        ++p;
        return true;
    }
    bool val(JVal &v) {
        ws();
        if (p >= e) return false;
        if (*p == '{') {
            v.t = JVal::OBJ;
            ++p;
            ws();
            if (p < e && *p == '}') { ++p; return true; }
            for (;;) {
                ws();
                std::string k;
                if (!str(k)) return false;
                ws();
                if (p >= e || *p != ':') return false;
                ++p;
                JVal c;
                if (!val(c)) return false;
                v.obj.emplace_back(std::move(k), std::move(c));
                ws();
                if (p < e && *p == ',') { ++p; continue; }
                if (p < e && *p == '}') { ++p; return true; }
                return false;
            }
        }
        if (*p == '[') {
            v.t = JVal::ARR;
            ++p;
            ws();
            if (p < e && *p == ']') { ++p; return true; }
            for (;;) {
                JVal c;
                if (!val(c)) return false;
                v.arr.push_back(std::move(c));
                ws();
                if (p < e && *p == ',') { ++p; continue; }
                if (p < e && *p == ']') { ++p; return true; }
                return false;
            }
        }
        if (*p == '"') { v.t = JVal::STR; return str(v.str); }
        if (*p >= '0' && *p <= '9') {
            v.t = JVal::NUM;
            v.num = strtoull(p, (char **)&p, 10);
            return true;
        }
        while (p < e && *p != ',' && *p != '}' && *p != ']') ++p;  // null / true / false / negative
        v.t = JVal::OTHER;
        return true;
    }
};

bool is_vendor_wrapper(const std::string &tag) {
    if (tag.size() <= 5 || tag.compare(tag.size() - 5, 5, "Error") != 0) return false;
    return vendor_pen(tag.substr(0, tag.size() - 5)) != 0;
}

// IE of a FieldSpecifier / ScopeFieldSpecifier element_id JSON value
void ie_from_json(const JVal &ie, ngz_error &out) {
    if (ie.t == JVal::STR) {
        if (const IeRow *r = ie_find_name(nullptr, ie.str)) out.ie_id = r->id;
        static const char *scope[] = {"System", "Interface", "LineCard", "Cache", "Template"};
        for (uint16_t i = 0; i < 5; ++i)
            if (ie.str == scope[i]) out.ie_id = (uint16_t)(i + 1);
        return;
    }
    if (ie.t != JVal::OBJ || ie.obj.size() != 1) return;
    const std::string &k = ie.obj[0].first;
    const JVal &v = ie.obj[0].second;
    if (k == "Unknown") {
        out.ie_pen = (uint32_t)v.u("pen");
        out.ie_id = (uint16_t)v.u("id");
        return;
    }
    out.ie_pen = vendor_pen(k);
    if (v.t == JVal::STR) {
        if (const IeRow *r = ie_find_name(k.c_str(), v.str)) out.ie_id = r->id;
    } else if (const JVal *u = v.get("Unknown")) {
        out.ie_id = (uint16_t)u->u("id");
    }
}

}  // namespace

extern "C" int ngz_dgram_error(ngz_ctx *ctx, uint32_t dgram, ngz_error *err) {
    if (!ctx || !err) return NGZ_E_INVALID;
    memset(err, 0, sizeof *err);
    err->field = 0xFFFF;
    const int n = ngz_dgram_error_json(ctx, dgram, nullptr, 0);
    if (n <= 0) return NGZ_E_INVALID;
    std::string text((size_t)n + 1, '\0');
    ngz_dgram_error_json(ctx, dgram, &text[0], text.size());
    text.resize((size_t)n);
    JVal root;
    JParse jp{text.data(), text.data() + text.size()};
    if (!jp.val(root)) return NGZ_E_INVALID;
    // walk the single-key enum wrappers down to the innermost variant (no
    // reference error variant is a struct of exactly one field)
    std::vector<std::string> tags;
    const JVal *v = &root;
    while (v->t == JVal::OBJ && v->obj.size() == 1) {
        tags.push_back(v->obj[0].first);
        v = &v->obj[0].second;
    }
    if (tags.empty()) return NGZ_E_INVALID;
    const std::string &kind = tags.back();
    bool record = false, tmpl = false, set = false, msg = false;
    for (const auto &t : tags) {
        if (t == "DataRecordError") record = true;
        if (t == "TemplateRecordError" || t == "OptionsTemplateRecordError" || t == "FieldSpecifierError" ||
            t == "ScopeFieldSpecifierError" || t == "IEError")
            tmpl = true;
        if (t == "SetParsingError" || t == "SetError") set = true;
        if (t == "IpfixParsingError" || t == "NetFlowV9ParingError") msg = true;
        if (is_vendor_wrapper(t)) err->vendor = 1;
    }
    err->layer = record ? NGZ_ERRL_RECORD : tmpl ? NGZ_ERRL_TEMPLATE : set ? NGZ_ERRL_SET
               : msg ? NGZ_ERRL_MESSAGE : NGZ_ERRL_CODEC;
    err->offset = (uint32_t)v->u("offset");
    if (kind == "UnsupportedVersion") {
        err->kind = NGZ_ERR_UNSUPPORTED_VERSION;
        err->value = v->t == JVal::NUM ? v->num : v->u("version");
    } else if (kind == "InvalidLength") {
        err->kind = NGZ_ERR_INVALID_LENGTH;
        if (v->t == JVal::ARR && v->arr.size() == 2) {  // FieldSpecifierError::InvalidLength(length, IE)
            err->length = (uint32_t)v->arr[0].num;
            ie_from_json(v->arr[1], *err);
        } else {
            err->length = (uint32_t)v->u("length");
            if (const JVal *ie = v->get("ie")) ie_from_json(*ie, *err);  // ScopeFieldSpecifier InvalidLength
        }
    } else if (kind == "UnexpectedEof") {
        err->kind = NGZ_ERR_UNEXPECTED_EOF;
        err->length = (uint32_t)v->u("needed");
        err->available = (uint32_t)v->u("available");
    } else if (kind == "InvalidPaddingLength") {
        err->kind = NGZ_ERR_INVALID_PADDING_LENGTH;
        err->length = (uint32_t)v->u("requested");
        err->value = v->u("ret_len");
    } else if (kind == "InvalidSetId") {
        err->kind = NGZ_ERR_INVALID_SET_ID;
        err->value = v->u("id");
    } else if (kind == "NoTemplateDefinedFor") {
        err->kind = NGZ_ERR_NO_TEMPLATE;
        err->value = v->u("id");
    } else if (kind == "InvalidPaddingValue") {
        err->kind = NGZ_ERR_INVALID_PADDING_VALUE;
        err->value = v->u("value");
    } else if (kind == "InvalidCount") {
        err->kind = NGZ_ERR_INVALID_COUNT;
        err->value = v->u("count");
    } else if (kind == "InvalidTemplateId") {
        err->kind = NGZ_ERR_INVALID_TEMPLATE_ID;
        err->value = v->u("template_id");
    } else if (kind == "InvalidScopeFieldsCount") {
        err->kind = NGZ_ERR_INVALID_SCOPE_FIELDS_COUNT;
        err->value = v->u("scope_fields_count");
        err->length = (uint32_t)v->u("total_fields_count");
    } else if (kind == "UndefinedIANAIE") {
        err->kind = NGZ_ERR_UNDEFINED_IANA_IE;
        err->ie_id = (uint16_t)(v->t == JVal::NUM ? v->num : 0);
    } else if (kind == "InvalidTimestamp") {
        err->kind = NGZ_ERR_INVALID_TIMESTAMP;
        err->value = v->u("seconds");
    } else if (kind == "InvalidTimestampMillis") {
        err->kind = NGZ_ERR_INVALID_TIMESTAMP_MILLIS;
        err->value = v->u("millis");
    } else if (kind == "InvalidTimestampFraction") {
        err->kind = NGZ_ERR_INVALID_TIMESTAMP_FRACTION;
        err->value = v->u("seconds");
        err->length = (uint32_t)v->u("fraction");
    } else if (kind == "Utf8Error") {
        err->kind = NGZ_ERR_UTF8;
    } else {
        return NGZ_E_INVALID;
    }
    if (record) {
        // the failing field: index `a` of a device record error key, or the
        // IE named in the error for host-framed datagrams
        ngz_dgram_hdr h;
        if (hipMemcpy(&h, ctx->d_hdr.p + dgram, sizeof h, hipMemcpyDeviceToHost) != hipSuccess) return NGZ_E_DEVICE;
        h.err_key = record_err_key(ctx, dgram, h.err_key);
        const uint32_t code = (uint32_t)(h.err_key >> 40) & 0xFF;
        if (code >= E_REC_DTMS && code <= E_REC_EOF && code != E_HOST) {
            const uint32_t stop = (uint32_t)(h.err_key >> 48);
            const uint32_t f = (uint32_t)(h.err_key >> 24) & 0xFFFF;
            // the version of the set holding the stop position
            std::vector<ngz_set_info> sets(ctx->summary.n_sets);
            if (!sets.empty() &&
                hipMemcpy(sets.data(), ctx->d_sets.p, sets.size() * sizeof(ngz_set_info), hipMemcpyDeviceToHost) !=
                    hipSuccess)
                return NGZ_E_DEVICE;
            for (const auto &si : sets) {
                if (si.dgram != dgram || si.set_pos >= stop) continue;
                const Version &ver = ctx->versions[ctx->slot_version[si.slot]];
                if (f < ver.specs.size()) {
                    err->field = (uint16_t)f;
                    err->ie_pen = ver.specs[f].pen;
                    err->ie_id = ver.specs[f].id;
                }
            }
        }
    }
    return NGZ_OK;
}
