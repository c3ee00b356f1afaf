// Host-side internals shared by ngz_host.cpp (C ABI, template registry,
// batch pipeline), ngz_json.cpp (serde-JSON rendering of decoded datagrams)
// and ngz_collector.cpp (per-peer stream framing, pcap/UDP ingest).  Not part
// of the C ABI.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <map>
#include <vector>

#include "ngz/flow_aggregate.h"
#include "ngz/flow_decode.h"
#include "ngz_internal.h"

// NGZ_OPT_SPECIALIZE 2: a template's kernel is compiled once it has decoded this many records
#define NGZ_SPECIALIZE_MIN_RECORDS 65536
#define NGZ_MAX_AUX 7  // auxiliary decode streams per context

namespace ngzh {

// ------------------------------------------------------------------------
// IE registry rows (generated from the reference XML, tools/gen_ie_registry.py)
// ------------------------------------------------------------------------
enum DataType : uint8_t {
    DT_octetArray = 0, DT_unsigned8, DT_unsigned16, DT_unsigned32, DT_unsigned64, DT_signed8, DT_signed16,
    DT_signed32, DT_signed64, DT_float32, DT_float64, DT_boolean, DT_macAddress, DT_string, DT_dateTimeSeconds,
    DT_dateTimeMilliseconds, DT_dateTimeMicroseconds, DT_dateTimeNanoseconds, DT_ipv4Address, DT_ipv6Address,
    DT_basicList, DT_subTemplateList, DT_subTemplateMultiList, DT_unsigned256,
};

struct IeRow {
    uint32_t pen;
    uint16_t id;
    uint8_t dtype;
    uint8_t flags;  // 1 mpls, 2 tcpControlBits, 4 sub-registry
    const char *name;
};
struct VendorRow {
    uint32_t pen;
    const char *name;
};

// (pen, id) -> registry row, or null
const IeRow *ie_find(uint32_t pen, uint16_t id);
// (vendor display name or null for IANA, IE name) -> registry row, or null
const IeRow *ie_find_name(const char *vendor, const std::string &name);
// vendor display name -> PEN (0 if unknown)
uint32_t vendor_pen(const std::string &vendor);
// vendor display name of a PEN with its own IE package, or null
const char *vendor_name(uint32_t pen);
// sub-registry of an IE: 0 none, 1 value-name enum, 2 nested reason codes (ngz_json.cpp)
int subreg_kind(uint32_t pen, uint16_t id);
// is v a registered variant of the IE's sub-registry enum
bool subreg_known(uint32_t pen, uint16_t id, uint64_t v);
// ranks of values 0..255 (+ [256] for larger ones) in the Ord of a nested sub-registry's enum (ngz_json.cpp)
bool subreg_nested_ranks(uint32_t pen, uint16_t id, uint64_t rank[257]);

// ------------------------------------------------------------------------
// Template model
// ------------------------------------------------------------------------
enum IeKind : uint8_t { IK_IANA, IK_VENDOR, IK_VENDOR_UNKNOWN, IK_UNKNOWN, IK_SCOPE };

struct Spec {
    IeKind kind;
    uint8_t dtype;
    uint8_t flags;
    bool scope;
    uint32_t pen;
    uint16_t id;  // scope: raw code
    uint16_t length;
    const char *name;    // IANA/vendor IE name
    const char *vendor;  // vendor display name
};

struct Version {
    uint8_t proto = 0;  // 10 / 9
    uint16_t tid = 0;
    std::vector<Spec> specs;  // scope first
    uint32_t n_scope = 0;
    DevPlan plan{};                 // plan.f points into `fields` (re-pointed on copy / move)
    std::vector<DevField> fields;   // one descriptor per spec
    std::vector<uint8_t> fail_sub;  // per field: 1 InvalidLength, 2 InvalidPaddingLength, 3 scope InvalidLength
    uint64_t processed = 0;
    uint64_t seen_records = 0;      // records decoded with this version (NGZ_OPT_SPECIALIZE 2)
    int rtc_state = 0;              // specialised kernel: 0 not looked up, 1 ready, 2 unavailable, 3 compiling
    void *rtc_fn = nullptr;
    void *rtc_entry = nullptr;      // process-wide kernel cache entry (ngz_rtc.cpp), polled while compiling

    Version() = default;
    Version(const Version &o) { *this = o; }
    Version(Version &&o) noexcept { *this = std::move(o); }
    Version &operator=(const Version &o) {
        copy_scalars(o);
        specs = o.specs;
        fields = o.fields;
        fail_sub = o.fail_sub;
        plan.f = fields.data();
        return *this;
    }
    Version &operator=(Version &&o) noexcept {
        copy_scalars(o);
        specs = std::move(o.specs);
        fields = std::move(o.fields);
        fail_sub = std::move(o.fail_sub);
        plan.f = fields.data();
        return *this;
    }

  private:
    void copy_scalars(const Version &o) {
        proto = o.proto; tid = o.tid; n_scope = o.n_scope; plan = o.plan; processed = o.processed;
        seen_records = o.seen_records; rtc_state = o.rtc_state; rtc_fn = o.rtc_fn; rtc_entry = o.rtc_entry;
    }
};

// serde_json helpers (ngz_host.cpp)
std::string json_str(const char *s);
std::string ie_json(const Spec &s);    // IE / ScopeIE element_id value
std::string spec_json(const Spec &s);  // FieldSpecifier / ScopeFieldSpecifier
std::string wrap(const char *tag, const std::string &inner);

inline uint32_t rd16(const uint8_t *p) { return ((uint32_t)p[0] << 8) | p[1]; }
inline uint32_t rd32(const uint8_t *p) {
    return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}

struct ErrInfo {  // host-side framing error
    std::string json;
};

// ------------------------------------------------------------------------
// Context
// ------------------------------------------------------------------------
template <class T>
struct DevBuf {
    T *p = nullptr;
    size_t cap = 0;
    bool contiguous = false;  // ask for physically contiguous memory (falls back to hipMalloc)
    int ensure(size_t n) {
        if (n <= cap) return 0;
        if (p) hipFree(p);
        p = nullptr;
        size_t c = std::max(n, cap + cap / 2);
        if (contiguous) {  // an experiment knob (NGZ_ARENA_CONTIG): say what was granted
            const bool ok = hipExtMallocWithFlags((void **)&p, c * sizeof(T) + 64, hipDeviceMallocContiguous) == hipSuccess;
            fprintf(stderr, "[ngz] contiguous allocation of %zu bytes: %s\n", c * sizeof(T) + 64, ok ? "granted" : "refused");
            if (ok) {
                cap = c;
                return 0;
            }
        }
        p = nullptr;
        if (hipMalloc((void **)&p, c * sizeof(T) + 64) != hipSuccess) {
            cap = 0;
            return -1;
        }
        cap = c;
        return 0;
    }
    void release() {
        if (p) hipFree(p);
        p = nullptr;
        cap = 0;
    }
};

// serde JSON of one (options) template set of a host-framed datagram
// ({"Template":[..]} / {"OptionsTemplate":[..]}), kept for the JSON renderer
struct TemplateSetJson {
    uint32_t dgram;
    uint32_t set_pos;
    std::string json;
};

// Host copies of one decoded batch for the JSON renderer (ngz_json.cpp)
struct JsonView {
    uint64_t serial = 0;                     // ngz_ctx::batch_serial it was loaded from
    std::vector<ngz_dgram_hdr> hdr;
    std::vector<ngz_set_info> sets;
    std::vector<uint32_t> set_first;         // CSR: data sets of datagram d
    std::vector<uint32_t> tset_first;        // CSR: ngz_ctx::tmpl_sets of datagram d
    std::vector<std::vector<uint8_t>> cols;  // per slot: its column block (slots with records)
    std::vector<uint8_t> own_bytes;          // D2H copy of the batch bytes when no host copy is given
    const uint8_t *bytes = nullptr;          // batch bytes (host)
    std::vector<uint64_t> offs;
    std::vector<uint32_t> lens;
    // ngz_record_fields: record offsets (in the datagram) of variable-length data sets, by set
    // index, walked on first use
    std::map<uint32_t, std::vector<uint32_t>> rec_pos;
};

}  // namespace ngzh

struct ngz_ctx;
struct ngz_agg;
namespace ngzh {
// aggregator internals the FlowInfo renderer reads (ngz_agg.hip)
const std::vector<ngz_agg_field> &agg_keys(const ngz_agg *a);
const std::vector<ngz_agg_field> &agg_vals(const ngz_agg *a);
void agg_out_dicts(const ngz_agg *a, const std::vector<int64_t> **t, const std::vector<int64_t> **p,
                   const std::vector<int64_t> **d);
const std::vector<ngz_peer> &agg_out_peers(const ngz_agg *a);
uint64_t agg_window_ms(const ngz_agg *a);
// Host template state of a context (both TemplatesMaps): saved before a
// speculative batch and restored when its framing guess was wrong (ngz_collector.cpp)
struct TemplateState {
    std::vector<Version> versions;
    std::vector<int32_t> cur[2];
};
void state_save(ngz_ctx *ctx, TemplateState &s);
// a datagram's error key as the reference reports it (a value error before a walk's failure, ngz_host.cpp)
uint64_t record_err_key(ngz_ctx *ctx, uint32_t dgram, uint64_t key);
void state_restore(ngz_ctx *ctx, const TemplateState &s);
// D2H of the last batch (host_bytes: the batch bytes already in host memory, or null)
int json_view_load(ngz_ctx *ctx, const uint8_t *host_bytes, JsonView &v);
// serde JSON of datagram d (FlowInfo, or the error) appended to `out`; returns its
// NGZ_DG_* status and the bytes FlowInfoCodec::decode consumed from it
// (codec.rs:151-183: IPFIX length, NFv9 end of the last parsed set, errors per the codec)
int json_render(ngz_ctx *ctx, const JsonView &v, uint32_t d, std::string &out, uint32_t *consumed);
}  // namespace ngzh

struct ngz_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    std::string last_error;
    std::vector<ngzh::Version> versions;              // append-only
    std::vector<int32_t> cur[2];                // [proto idx][template id] -> version or -1
    // batch
    std::vector<int32_t> slot_version;          // slot -> version
    std::vector<int32_t> version_slot;          // version -> slot (this batch) or -1
    ngzh::DevBuf<DevPlan> d_plans;
    ngzh::DevBuf<DevField> d_fields;             // field tables of the uploaded plans (DevPlan::f)
    ngzh::DevBuf<uint16_t> d_cur_slot;
    ngzh::DevBuf<uint32_t> d_tl_key, d_tl_dgram;
    ngzh::DevBuf<uint16_t> d_tl_slot;
    ngzh::DevBuf<uint32_t> d_hf_flag;
    ngzh::DevBuf<ngz_dgram_hdr> d_hf_hdr;
    ngzh::DevBuf<uint32_t> d_hf_first;
    ngzh::DevBuf<HostSet> d_hf_sets;
    ngzh::DevBuf<ngz_dgram_hdr> d_hdr;
    ngzh::DevBuf<uint32_t> d_counts, d_scan;
    ngzh::DevBuf<uint8_t> d_scan_tmp;
    ngzh::DevBuf<SlotRT> d_slots;
    ngzh::DevBuf<Chunk> d_chunks;
    ngzh::DevBuf<ngz_set_info> d_sets;
    ngzh::DevBuf<uint8_t> d_arena;
    ngzh::DevBuf<unsigned long long> d_proc;
    ngzh::DevBuf<BatchSummary> d_summary;
    ngzh::DevBuf<uint32_t> d_recmap;            // record-start bitmap of variable-length sets
    ngzh::DevBuf<uint16_t> d_recoff;            // per-datagram record-offset lists of variable-length sets
    ngzh::DevBuf<unsigned long long> d_dsum;    // per datagram: its one data set (k_frame -> k_emit)
    // host staging for ngz_decode_batch_host
    ngzh::DevBuf<uint8_t> d_in_bytes;
    ngzh::DevBuf<uint64_t> d_in_off;
    ngzh::DevBuf<uint32_t> d_in_len;
    // results of the last batch
    std::vector<ngz_slot_info> slot_infos;
    std::vector<SlotRT> slot_rt;
    std::vector<ngzh::ErrInfo> host_errors;
    BatchSummary summary{};
    ngz_batch_in last_in{};
    hipEvent_t ev[4]{};
    // auxiliary decode streams: per-template kernels of one batch run side by side
    uint32_t n_aux = 0;                         // NGZ_DECODE_STREAMS - 1 (side-by-side decode measured no better:
                                                //  config 3 4.34 vs 4.42 ms, config 4 1.95 vs 2.40 ms serial vs 4 streams)
    hipStream_t aux[NGZ_MAX_AUX]{};
    hipEvent_t join_ev[NGZ_MAX_AUX]{};
    hipEvent_t fork_ev = nullptr;
    int n_cus = 256;
    int specialize = 1;                         // NGZ_OPT_SPECIALIZE
    bool rtc_sync = false;                      // NGZ_OPT_RTC_SYNC: wait for a template's kernel compile
    std::vector<uint8_t> slot_spec;             // last batch: slot decoded by its specialised kernel
    uint32_t blocks_per_cu = 4;                 // decode grid: 4 x 256 threads per CU
    uint32_t lds_blocks_per_cu = 8;             // LDS-staged decode grid (2 resident per CU at 64 KB)
    // multi-template decode launches (ngz_rtc.cpp generate_group): one kernel for the
    // LDS-staged specialised templates of a batch that share a workgroup shape, per set of
    // template versions; NGZ_OPT_GROUP 1 turns it on (default: one launch per template)
    struct GroupKernel {
        int state = 0;  // 0 not looked up, 1 ready, 2 unavailable, 3 compiling
        void *fn = nullptr;
        void *entry = nullptr;
    };
    std::map<std::vector<int32_t>, GroupKernel> group_kernels;
    bool group_launch = false;                  // NGZ_OPT_GROUP
    int split_framing = 0;                      // NGZ_OPT_SPLIT
    // device summary / processed_count increments alternate between two
    // parities: a batch's k_export zeroes the other parity for the next one
    int parity = 0;
    bool clean[2] = {false, false};
    uint64_t assigned_gen = 0;                  // tmpl_gen the slot assignment was computed for
    BatchSummary *h_summary = nullptr;          // pinned
    SlotRT *h_slots = nullptr;                  // pinned, NGZ_MAX_SLOTS
    unsigned long long *h_proc = nullptr;       // pinned, NGZ_MAX_SLOTS: processed_count increments
    BatchSummary *dh_summary = nullptr;         // device aliases of the three pinned export buffers
    SlotRT *dh_slots = nullptr;
    unsigned long long *dh_proc = nullptr;
    unsigned long long *h_done = nullptr, *dh_done = nullptr;  // k_export completion word (pinned)
    unsigned long long export_seq = 0;
    uint32_t cap_pad_windows = 0;               // NGZ_OPT_CAP_PAD
    int place_trials = 6;                       // arena placement trials on the first large batch (NGZ_OPT_PLACE_TRIALS)
    bool placed = false;
    std::vector<float> place_ms;                // decode ms of each placement trial (ngz_placement_trials)
    std::vector<float> place_probe_ms;          // probe ms of each trial (NGZ_OPT_PLACE_PROBE)
    int place_probe = 0;                        // NGZ_OPT_PLACE_PROBE
    uint32_t place_kept = 0;                    // the trial whose arena was kept
    // ngz_decode_batch_submit / _wait: the context's decode worker, started on first use
    struct AsyncDecode {
        std::thread th;
        std::mutex m;
        std::condition_variable cv;
        bool job = false;     // a submitted batch the worker has not finished
        bool result = false;  // a finished batch whose result the host has not collected
        bool stop = false;
        std::atomic<bool> pending{false};  // job || result: other calls on the context are refused
        ngz_batch_in in{};
        ngz_batch_out *out = nullptr;
        void *stream = nullptr;
        int rc = 0;
    } async;
    uint64_t arena_shift = 0;                   // NGZ_OPT_ARENA_SHIFT: columns start this far into the arena
    bool spin_wait = true;                      // wait for a batch by spinning on h_done (NGZ_SPIN=0: stream sync)
    float t_decode = 0, t_pipeline = 0;
    bool plans_dirty = true;
    uint32_t n_template_dgrams = 0;
    uint64_t tmpl_gen = 1, uploaded_gen = 0;  // template-state generation vs the device tables
    // steady-state decode launches (run_pipeline): the slots of the last batch
    bool pred_valid = false;
    std::vector<int32_t> pred_versions;
    std::vector<uint8_t> pred_active;
    // count-matrix rows (BatchDev::slot_row): the slots of the last batch, or every slot (first
    // batch after a template change, host-framed batches, and the retry of a batch that met a
    // slot without a row)
    bool rows_all = false;
    std::vector<uint16_t> slot_row_host;  // what d_slot_row holds
    ngzh::DevBuf<uint16_t> d_slot_row;
    // split framing (run_pipeline): phase B's count matrix, scan and rows (the variable-length
    // slots), its stream and fork / join events; split_skip: batches left without splitting after
    // phase B met a record error
    ngzh::DevBuf<uint32_t> d_counts2, d_scan2;
    ngzh::DevBuf<uint8_t> d_scan_tmp2;
    ngzh::DevBuf<uint16_t> d_slot_row2;
    std::vector<uint16_t> slot_row2_host;
    hipStream_t split_stream = nullptr;
    hipEvent_t split_ev[3] = {};
    uint32_t split_skip = 0;
    uint32_t batch_info = 0, pipeline_runs = 0;  // ngz_last_batch_info
    ngzh::DevBuf<unsigned long long> d_trace;  // NGZ_TRACE window clocks
    hipEvent_t d2h_ev = nullptr;  // ngz_columns_to_host_async: the last queued copy of the columns
    bool d2h_pending = false;
    std::vector<ngzh::TemplateSetJson> tmpl_sets;  // template sets of the last batch, (dgram, set_pos) order
    // versions re-announced (identically) in this batch -> (datagram << 16 | template record position)
    // of the last re-announcement: processed_count restarts there (DevPlan::count_from)
    std::map<int32_t, uint64_t> count_from;
    uint64_t batch_serial = 0;                      // bumped by every ngz_decode_batch
    std::shared_ptr<ngzh::JsonView> json_view;      // ngz_dgram_json cache of the last batch
    // ngz_template_counts_device staging: a ring of pinned tables, each reused only after
    // the copy that last read it has completed (its event), so no call waits on the copy
    // it or the previous call just queued
    static constexpr int COUNTS_RING = 4;
    uint64_t *h_counts_stage[COUNTS_RING] = {};
    uint32_t h_counts_cap[COUNTS_RING] = {};
    hipEvent_t counts_ev[COUNTS_RING] = {};
    uint32_t counts_next = 0;
};
