// ngz-pcap-decoder: the reference's `pcap-decoder --protocol flow` command line
// (crates/pcap-decoder/src/main.rs:23-95) over the MI355X decoder
// (ngz_pcap_to_jsonl, include/ngz/flow_ingest.h).  Same flags and output;
// only the flow protocol is built in this repository.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "ngz/flow_ingest.h"

static void usage(const char *argv0) {
    fprintf(stderr,
            "usage: %s -i <INPUT> [-o <OUTPUT>] --protocol flow --ports <PORTS> [-c <INPUT_COUNT>] "
            "[--show-frame-number] [--device <N>]\n",
            argv0);
}

int main(int argc, char **argv) {
    const char *input = nullptr, *output = nullptr, *protocol = nullptr;
    std::vector<uint16_t> ports;
    int64_t count = -1;
    int frames = 0, device = 0;
    for (int i = 1; i < argc; ++i) {
        std::string a = argv[i];
        std::string val;
        const size_t eq = a.find('=');
        if (a.rfind("--", 0) == 0 && eq != std::string::npos) {
            val = a.substr(eq + 1);
            a = a.substr(0, eq);
        }
        auto next = [&]() -> const char * {
            if (!val.empty()) return strdup(val.c_str());
            if (i + 1 >= argc) { usage(argv[0]); exit(2); }
            return argv[++i];
        };
        if (a == "-i" || a == "--input") input = next();
        else if (a == "-o" || a == "--output") output = next();
        else if (a == "--protocol") protocol = next();
        else if (a == "--ports") {  // comma-separated (value_delimiter = ',')
            std::string s = next();
            size_t at = 0;
            while (at <= s.size()) {
                const size_t c = s.find(',', at);
                const std::string tok = s.substr(at, c == std::string::npos ? std::string::npos : c - at);
                if (!tok.empty()) ports.push_back((uint16_t)atoi(tok.c_str()));
                if (c == std::string::npos) break;
                at = c + 1;
            }
        } else if (a == "-c" || a == "--input-count") count = atoll(next());
        else if (a == "--show-frame-number") frames = 1;
        else if (a == "--device") device = atoi(next());
        else if (a == "-h" || a == "--help") { usage(argv[0]); return 0; }
        else { fprintf(stderr, "unexpected argument '%s'\n", a.c_str()); usage(argv[0]); return 2; }
    }
    if (!input || !protocol || ports.empty()) { usage(argv[0]); return 2; }
    if (ngz_abi_version() != NGZ_ABI_VERSION) {
        fprintf(stderr, "ngz-pcap-decoder: libngz ABI %d, built against %d\n", ngz_abi_version(), NGZ_ABI_VERSION);
        return 2;
    }
    std::string p = protocol;
    for (auto &ch : p) ch = (char)tolower(ch);
    if (p != "flow") {
        fprintf(stderr, "protocol '%s': only `flow` (IPFIX / NetFlow v9) is built in netgauze_amd\n", protocol);
        return 2;
    }
    const int64_t n = ngz_pcap_to_jsonl(input, ports.data(), (uint32_t)ports.size(), output, device, count, frames);
    if (n < 0) {
        fprintf(stderr, "ngz-pcap-decoder: failed (%lld)\n", (long long)n);
        return 1;
    }
    return 0;
}
