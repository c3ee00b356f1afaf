// Host check of ngz_vlen_walk (fast walk program) against ngz_vlen_walk_exact
// (one step per field) on random variable-length records with random
// truncation and corruption: same record count, record offsets and error key.
// Built and run by tests/test_vlen_walk_host.py (hipcc, host code only).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#include "../../netgauze_amd/csrc/ngz_internal.h"

int main() {
    std::mt19937_64 rng(12345);
    long fails = 0, cases = 0, errors = 0;
    for (int t = 0; t < 4000; ++t) {
        // a random template: fixed fields (some DTFRAC) and up to 6 vlen fields
        const int nf = 1 + rng() % 12;
        std::vector<DevField> fs(nf);
        for (auto &f : fs) {
            memset(&f, 0, sizeof f);
            const int r = rng() % 6;
            if (r == 0) { f.kind = NGZ_K_VLEN; f.len = 0xFFFF; }
            else if (r == 1) { f.kind = NGZ_K_DTFRAC; f.len = 8; }
            else { f.kind = NGZ_K_UINT; f.len = 1 + rng() % 9; }
        }
        DevPlan P;
        memset(&P, 0, sizeof P);
        P.n_fields = (uint16_t)nf;
        P.f = fs.data();
        uint32_t k = 0, acc = 0, rl = 0;
        for (auto &f : fs) {
            rl += f.kind == NGZ_K_VLEN ? 1 : f.len;
            if (f.kind == NGZ_K_VLEN) { P.walk_fixed[k++] = (uint16_t)acc; acc = 0; }
            else acc += f.len;
        }
        P.walk_fixed[k] = (uint16_t)acc;
        P.walk_nv = (uint8_t)k;
        P.rec_len = rl;
        // a set of records, then truncate / corrupt
        std::vector<uint8_t> b(16, 0xAA);
        const int nrec = rng() % 20;
        for (int r = 0; r < nrec; ++r)
            for (auto &f : fs) {
                if (f.kind == NGZ_K_VLEN) {
                    uint32_t L = rng() % 8 == 0 ? 255 + rng() % 300 : rng() % 40;
                    if (L >= 255) { b.push_back(255); b.push_back((uint8_t)(L >> 16)); b.push_back((uint8_t)(L >> 8)); b.push_back((uint8_t)L); }
                    else b.push_back((uint8_t)L);
                    for (uint32_t i = 0; i < L; ++i) b.push_back((uint8_t)rng());
                } else {
                    for (uint32_t i = 0; i < f.len; ++i) b.push_back((uint8_t)rng());
                }
            }
        uint32_t end = (uint32_t)b.size();
        if (rng() % 2 && end > 16) end = 16 + rng() % (end - 16 + 1);           // truncated set
        if (rng() % 4 == 0 && end > 16) b[16 + rng() % (end - 16)] = (uint8_t)rng();  // corrupted byte
        b.resize(end + 8, 0);
        std::vector<uint32_t> ra, rb;
        uint64_t ea = NGZ_NO_ERR, eb = NGZ_NO_ERR;
        const uint32_t na = ngz_vlen_walk(b.data(), 16, end, P, &ea, [&](uint32_t i, uint32_t at) { ra.push_back(i << 20 | at); });
        const uint32_t nb = ngz_vlen_walk_exact(b.data(), 16, end, P, &eb, [&](uint32_t i, uint32_t at) { rb.push_back(i << 20 | at); });
        ++cases;
        errors += eb != NGZ_NO_ERR;
        if (na != nb || ea != eb || ra != rb) {
            if (fails++ < 5) printf("mismatch case %d: n %u/%u err %llx/%llx\n", t, na, nb, (unsigned long long)ea, (unsigned long long)eb);
        }
    }
    printf("cases %ld errors %ld mismatches %ld\n", cases, errors, fails);
    return fails ? 1 : 0;
}
